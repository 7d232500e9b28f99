#!/bin/bash
# GPU parity + sampler files, then probe_classes at a given chain count alternating run-time settings.
# Usage: ab_env_c_parity.sh <tag> <chains> "ENV=a" ...
set -o pipefail
TAG=$1; C=$2; shift 2
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_scale_parity.py tests/test_gpu_sampler.py \
    tests/test_gpu_api.py -x -q --timeout 300 --timeout-method thread > gpurun_out/${TAG}_parity.txt 2>&1 && \
bash profiles/scripts/ab_env_c.sh $TAG $C "$@"
