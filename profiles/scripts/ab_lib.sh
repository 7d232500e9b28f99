#!/bin/bash
# layer-backward build variants: GPU parity on the default library, then probe_classes alternating the default
# with each _var/<name>.so given, a kernel trace of the default and the phase stamps from _var/bbstamp.so.
# Usage: bash profiles/scripts/ab_lib.sh <tag> <variant> ...
set -o pipefail
mkdir -p gpurun_out
TAG=$1; shift
ARGS=("VIHMC_BWD_V2=2")
for v in "$@"; do ARGS+=("VIHMC_ALLOW_DIAG=1 VIHMC_LIB=$PWD/_var/$v.so"); done
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_scale_parity.py -x -q --timeout 300 \
    --timeout-method thread > gpurun_out/${TAG}_parity.txt 2>&1 && \
bash profiles/scripts/ab_env.sh $TAG "${ARGS[@]}" && \
bash profiles/scripts/ktrace.sh $TAG && \
VIHMC_ALLOW_DIAG=1 VIHMC_LIB=$PWD/_var/bbstamp.so timeout -k 10 120 python profiles/scripts/diag/stamps_bwd.py \
    > gpurun_out/${TAG}_stamps.log 2>&1
