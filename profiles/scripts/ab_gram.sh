#!/bin/bash
# A/B of Gram-form variant libraries: alternating probe runs (gradient-only evaluations, 16 chains) of the in-tree
# library and each _ab/<v>.so. Usage: bash profiles/scripts/ab_gram.sh <tag> <variant> [<variant> ...]
TAG=$1; shift
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
O=$ROOT/gpurun_out/${TAG}_ab.txt
: > $O
for rep in 1 2; do
  timeout -k 10 120 python3 $ROOT/profiles/scripts/probes/probe_classes.py --chains 16 --iters 20 --grad --tag base >> $O 2>&1 || exit 1
  for v in "$@"; do
    VIHMC_LIB=$ROOT/_ab/$v.so timeout -k 10 120 python3 $ROOT/profiles/scripts/probes/probe_classes.py --chains 16 --iters 20 --grad --tag $v >> $O 2>&1 || exit 1
  done
done
