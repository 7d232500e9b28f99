#!/bin/bash
# layer-backward variants: GPU parity files on the default, probe_classes alternating v2 / v1, a kernel trace, and
# the v2 phase stamps from _var/bbstamp.so (a -DBB_STAMP=1 build).
set -o pipefail
mkdir -p gpurun_out
TAG=${1:-r02s}
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_scale_parity.py -x -q --timeout 300 \
    --timeout-method thread > gpurun_out/${TAG}_parity.txt 2>&1 && \
bash profiles/scripts/ab_env.sh $TAG VIHMC_BWD_V2=2 VIHMC_BWD_V2=0 && \
bash profiles/scripts/ktrace.sh $TAG && \
VIHMC_ALLOW_DIAG=1 VIHMC_LIB=$PWD/_var/bbstamp.so timeout -k 10 120 python profiles/scripts/diag/stamps_bwd.py \
    > gpurun_out/${TAG}_stamps.log 2>&1
