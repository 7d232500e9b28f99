#!/bin/bash
# Quick GPU iteration (one gpurun call): focused parity tests + eval probe timing.
# Usage: bash profiles/scripts/probes/quick_gpu.sh [pytest -k expression]
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
K=${1:-"bf16x6 or geometry"}
cd $ROOT
timeout -k 10 400 python -m pytest tests -m gpu -x -q -s -k "$K" > gpurun_out/t.log 2>&1
rc=$?
tail -3 gpurun_out/t.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python profiles/scripts/probes/probe_eval.py --chains 1 16 --iters 30 > gpurun_out/probe.log 2>&1
