#!/bin/bash
# In-tree library vs a variant build (_ab/<name>.so) in one GPU call: probe_classes.py alternating three times.
# Usage: bash profiles/scripts/ab_so2.sh <tag> <chains> <variant.so>
TAG=$1; C=$2; V=$3
mkdir -p gpurun_out
for rep in 1 2 3; do
  timeout -k 10 120 python profiles/scripts/probes/probe_classes.py --chains $C --iters 30 --tag new \
      >> gpurun_out/${TAG}_ab.txt 2>/dev/null || exit 1
  VIHMC_LIB=$PWD/$V timeout -k 10 120 python profiles/scripts/probes/probe_classes.py --chains $C --iters 30 --tag old \
      >> gpurun_out/${TAG}_ab.txt 2>/dev/null || exit 1
done
