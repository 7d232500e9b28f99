#!/bin/bash
# Round 6: kernel trace of the one-chain legs (probe_legs.py: DeepONet one chain, config 4), summarised per
# evaluation phase (trace_summary.py).
TAG=${TAG:-r06bb}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $ROOT/gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d $ROOT/gpurun_out/${TAG}_kt -o t -- \
    python3 $ROOT/profiles/scripts/probes/probe_legs.py --reps 1 > $ROOT/gpurun_out/${TAG}_kt.log 2>&1 || exit 1
python3 $ROOT/profiles/scripts/diag/trace_summary.py $(ls $ROOT/gpurun_out/${TAG}_kt/*kernel_trace.csv | head -1) > $ROOT/gpurun_out/${TAG}_trace.txt 2>&1
cat $ROOT/gpurun_out/${TAG}_trace.txt; tail -3 $ROOT/gpurun_out/${TAG}_kt.log
