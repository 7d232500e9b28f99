#!/bin/bash
# A/B: the in-tree library vs _ab/<v>.so on the gradient-only probe (16 chains), alternating, 3 rounds.
TAG=$1; shift
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
O=$ROOT/gpurun_out/${TAG}_ab.txt
: > $O
for rep in 1 2 3; do
  timeout -k 10 120 python3 $ROOT/profiles/scripts/probes/probe_classes.py --chains 16 --iters 20 --grad --tag new >> $O 2>&1 || exit 1
  for v in "$@"; do
    VIHMC_LIB=$ROOT/_ab/$v.so timeout -k 10 120 python3 $ROOT/profiles/scripts/probes/probe_classes.py --chains 16 --iters 20 --grad --tag $v >> $O 2>&1 || exit 1
  done
done
