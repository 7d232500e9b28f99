#!/bin/bash
# GPU parity files, then probe_classes alternating run-time settings, then a kernel trace of the default.
# Usage: bash profiles/scripts/ab_env_parity.sh <tag> "ENV=a" "ENV=b" ...
set -o pipefail
mkdir -p gpurun_out
TAG=$1; shift
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_scale_parity.py tests/test_gpu_sampler.py -x -q \
    --timeout 300 --timeout-method thread > gpurun_out/${TAG}_parity.txt 2>&1 && \
bash profiles/scripts/ab_env.sh $TAG "$@" && \
bash profiles/scripts/ktrace.sh $TAG
