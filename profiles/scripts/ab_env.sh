#!/bin/bash
# A/B of run-time knobs in one GPU call: probe_classes.py per setting, alternating twice.
# Usage: bash profiles/scripts/ab_env.sh <tag> "ENV=a" "ENV=b" ...
TAG=$1; shift
mkdir -p gpurun_out
for rep in 1 2; do
  for kv in "$@"; do
    env $kv timeout -k 10 120 python profiles/scripts/probes/probe_classes.py --chains 16 --iters 30 --tag "$kv" \
        >> gpurun_out/${TAG}_ab.txt 2>/dev/null || exit 1
  done
done
