#!/bin/bash
# Config 4's end-point value evaluation on a side stream: the split / sampler tests, then probe_side.py (on / off
# alternating in one process).
TAG=${TAG:-r05sv}
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread -p no:cacheprovider \
    tests/test_gpu_split_fused.py tests/test_gpu_scale_parity.py tests/test_gpu_sampler.py tests/test_gpu_scripts.py \
    > gpurun_out/${TAG}_tests.txt 2>&1
rc=$?; tail -3 gpurun_out/${TAG}_tests.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u profiles/scripts/probes/probe_side.py 3 > gpurun_out/${TAG}_ab.txt 2>/dev/null || exit 1
cat gpurun_out/${TAG}_ab.txt
