#!/bin/bash
# Kernel trace of the evaluation probe at a given chain count (plan sized for it). Usage: ktrace_c.sh <tag> <chains>
TAG=$1; C=$2
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $ROOT/gpurun_out
timeout -k 10 120 python3 $ROOT/profiles/scripts/probes/probe_classes.py --chains $C --iters 30 --tag C$C > $ROOT/gpurun_out/${TAG}_probe.txt 2>&1 && \
cd /tmp && export TMPDIR=/tmp && \
timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d $ROOT/gpurun_out/${TAG}_kt -o t -- \
    python3 $ROOT/profiles/scripts/probes/probe_classes.py --chains $C --iters 5 > $ROOT/gpurun_out/${TAG}_kt.log 2>&1
