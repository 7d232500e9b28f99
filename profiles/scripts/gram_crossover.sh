#!/bin/bash
# Gradient-only evaluation time with the Gram form on / off at several chain counts (where does it start to pay?).
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
O=$ROOT/gpurun_out/${1:-g}_cross.txt
: > $O
for C in 1 2 4 8 12 16; do
  for g in 1 0; do
    timeout -k 10 120 python3 $ROOT/profiles/scripts/probes/probe_classes.py --chains $C --iters 20 --grad --opt gram=$g \
        --opt gram_min_chains=1 --tag "gram=$g" >> $O 2>&1 || exit 1
  done
done
