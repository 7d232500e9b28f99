#!/bin/bash
# Per-kernel times of A/B variant builds (make -C vi-hmc_amd OUT=_var/<name>.so BUILD=build/<name>
# EXTRA=-D...), one rocprofv3 --kernel-trace --stats pass per variant over the C=16 eval probe, one GPU
# call: bash profiles/ab_kstats.sh <tag> base <name>.so ...   ("base" = the in-tree build)
set -e
TAG=$1; shift
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
O=$ROOT/gpurun_out/$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
export VIHMC_ALLOW_DIAG=1   # timing-only ablation variants are timed here, never used for results
for f in "$@"; do
  if [ "$f" = base ]; then unset VIHMC_LIB; else export VIHMC_LIB=$ROOT/_var/$f; fi
  timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$f -o s -- \
      python3 $ROOT/profiles/scripts/probes/probe_eval.py --chains 16 --iters 20 > $O/$f.log 2>&1
  echo "== $f: $(grep 'C= 16' $O/$f.log)" >> $O/summary.txt
  python3 $ROOT/profiles/kstats.py $(ls $O/$f/*kernel_stats.csv | head -1) 8 >> $O/summary.txt
done
