#!/bin/bash
# Kernel trace of one evaluation sequence. Usage: ktrace_lib.sh <tag> <chains> [variant.so] [extra probe args]
TAG=$1; C=$2; V=$3; shift 3
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $ROOT/gpurun_out
if [ -n "$V" ]; then export VIHMC_LIB=$ROOT/$V VIHMC_ALLOW_DIAG=1; fi
cd /tmp && export TMPDIR=/tmp && \
timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d $ROOT/gpurun_out/${TAG}_kt -o t -- \
    python3 $ROOT/profiles/scripts/probes/probe_classes.py --chains $C --iters 5 "$@" > $ROOT/gpurun_out/${TAG}_kt.log 2>&1 && \
cd $ROOT && python3 profiles/ktrace_eval.py gpurun_out/${TAG}_kt > gpurun_out/${TAG}_eval.txt
