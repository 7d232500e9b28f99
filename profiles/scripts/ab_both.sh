#!/bin/bash
# A/B: in-tree library vs _ab/<v>.so on the full and the gradient-only probe (16 chains) and one chain, alternating.
TAG=$1; shift
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
O=$ROOT/gpurun_out/${TAG}_ab.txt
: > $O
P=$ROOT/profiles/scripts/probes/probe_classes.py
for rep in 1 2; do
  for v in new "$@"; do
    L=""; [ "$v" != new ] && L=$ROOT/_ab/$v.so
    VIHMC_LIB=$L timeout -k 10 120 python3 $P --chains 16 --iters 20 --grad --tag "$v grad" >> $O 2>&1 || exit 1
    VIHMC_LIB=$L timeout -k 10 120 python3 $P --chains 16 --iters 20 --tag "$v full" >> $O 2>&1 || exit 1
    VIHMC_LIB=$L timeout -k 10 120 python3 $P --chains 1 --iters 20 --tag "$v c1" >> $O 2>&1 || exit 1
  done
done
