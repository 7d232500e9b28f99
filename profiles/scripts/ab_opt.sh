#!/bin/bash
# A/B of plan options in one GPU call: probe_classes.py per setting, alternating three times.
# Usage: bash profiles/scripts/ab_opt.sh <tag> <chains> "" "key=v" "key=v key2=w" ...
TAG=$1; C=$2; shift 2
mkdir -p gpurun_out
for rep in 1 2 3; do
  for set in "$@"; do
    args=""
    for kv in $set; do args="$args --opt $kv"; done
    timeout -k 10 120 python profiles/scripts/probes/probe_classes.py --chains $C --iters 30 --tag "${set:-default}" $args \
        >> gpurun_out/${TAG}_ab.txt 2>/dev/null || exit 1
  done
done
