#!/bin/bash
# ab_lib.sh plus the sampler tests (fused DeepONet / BNN trajectories vs the step-by-step path and the CPU
# reference). Usage: bash profiles/scripts/ab_lib_sampler.sh <tag> <variant> ...
set -o pipefail
TAG=$1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_sampler.py -x -q --timeout 120 --timeout-method thread \
    > gpurun_out/${TAG}_sampler.txt 2>&1 && \
bash profiles/scripts/ab_lib.sh "$@"
