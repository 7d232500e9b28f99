#!/bin/bash
# probe_classes at a given chain count alternating run-time settings. Usage: ab_env_c.sh <tag> <chains> "ENV=a" ...
TAG=$1; C=$2; shift 2
mkdir -p gpurun_out
for rep in 1 2; do
  for kv in "$@"; do
    env $kv timeout -k 10 120 python profiles/scripts/probes/probe_classes.py --chains $C --iters 40 --tag "$kv" \
        >> gpurun_out/${TAG}_ab.txt 2>/dev/null || exit 1
  done
done
