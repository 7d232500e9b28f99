#!/bin/bash
# k_bwd_bf2 (staging waves) vs k_bwd_bf: parity file on v2, then probe_classes alternating, then a kernel trace.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_scale_parity.py -x -q --timeout 300 \
    --timeout-method thread > gpurun_out/r02l_parity.txt 2>&1 && \
bash profiles/scripts/ab_env.sh r02l VIHMC_BWD_V2=0 VIHMC_BWD_V2=1 && \
bash profiles/scripts/ktrace.sh r02l
