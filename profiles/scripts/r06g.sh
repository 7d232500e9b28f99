#!/bin/bash
# Round 6: two-chain T_t units (k_gram_b2, plan option gram_pair2) -- bitwise tests, gradient-only class A/B at 16
# chains (alternating), rocprofv3 kernel stats of both arms.
O=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out
TAG=${TAG:-r06g}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_gram.py -v -k "pair2 or deterministic or burgers_matches" \
    --timeout 200 --timeout-method thread > $O/${TAG}_tests.txt 2>&1 || exit 1
P=profiles/scripts/probes/probe_classes.py
for rep in 1 2 3; do
  for v in 1 0; do
    timeout -k 10 120 python -u $P --chains 16 --iters 20 --grad --opt gram_pair2=$v --tag "pair2=$v" >> $O/${TAG}_ab.txt 2>&1 || exit 1
  done
done
for v in 1 0 2; do
  (cd /tmp && export TMPDIR=/tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv \
      -d $O/${TAG}_prof$v -o s -- python3 $GRAFT_REPO_ROOT/$P --chains 16 --iters 20 --grad --opt gram_pair2=$v \
      > $O/${TAG}_prof$v.log 2>&1) || exit 1
  python3 profiles/kstats.py $(ls $O/${TAG}_prof$v/*kernel_stats.csv | head -1) 16 > $O/${TAG}_kstats$v.txt 2>&1
done
