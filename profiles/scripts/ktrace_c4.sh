#!/bin/bash
# Kernel trace of config 4's single-chain half-shard evaluation. Usage: ktrace_c4.sh <tag>
TAG=$1
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $ROOT/gpurun_out
timeout -k 10 120 python3 $ROOT/profiles/scripts/probes/probe_classes.py --chains 1 --iters 30 --config4 --tag c4 > $ROOT/gpurun_out/${TAG}_probe.txt 2>&1 && \
cd /tmp && export TMPDIR=/tmp && \
timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d $ROOT/gpurun_out/${TAG}_kt -o t -- \
    python3 $ROOT/profiles/scripts/probes/probe_classes.py --chains 1 --iters 5 --config4 > $ROOT/gpurun_out/${TAG}_kt.log 2>&1 && \
cd $ROOT && python3 profiles/ktrace_eval.py gpurun_out/${TAG}_kt > gpurun_out/${TAG}_eval.txt
