#!/bin/bash
# Kernel trace (per-dispatch durations) of the C=16 evaluation probe. Usage: bash profiles/scripts/ktrace.sh <tag> [ENV=v ...]
TAG=$1; shift
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $ROOT/gpurun_out
cd /tmp && export TMPDIR=/tmp
for kv in "$@"; do
  export $kv
done
timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d $ROOT/gpurun_out/${TAG}_kt -o t -- \
    python3 $ROOT/profiles/scripts/probes/probe_classes.py --chains 16 --iters 5 > $ROOT/gpurun_out/${TAG}_kt.log 2>&1
