#!/bin/bash
# BNN: GPU sampler + surface tests, then probe_bnn alternating run-time settings.
# Usage: bash profiles/scripts/ab_bnn.sh <tag> "ENV=a" "ENV=b" ...
set -o pipefail
mkdir -p gpurun_out
TAG=$1; shift
timeout -k 10 600 python -u -m pytest tests/test_gpu_sampler.py tests/test_gpu_surface.py tests/test_gpu_api.py -x -q \
    --timeout 300 --timeout-method thread > gpurun_out/${TAG}_bnn_tests.txt 2>&1 || exit 1
for rep in 1 2; do
  for kv in "$@"; do
    env $kv timeout -k 10 120 python profiles/scripts/probes/probe_bnn.py --tag "$kv" >> gpurun_out/${TAG}_bnn_ab.txt 2>/dev/null || exit 1
  done
done
