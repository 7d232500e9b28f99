#!/bin/bash
set -e
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_api.py tests/test_gpu_sampler.py -x -q --timeout 120 --timeout-method thread > $O/gather_parity.log 2>&1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/gather_new -o s -- python3 $R/profiles/scripts/probes/probe_eval.py --chains 16 --iters 30 > $O/gather_new.log 2>&1
VIHMC_LIB=$R/_var/gather16.so timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/gather_old -o s -- python3 $R/profiles/scripts/probes/probe_eval.py --chains 16 --iters 30 > $O/gather_old.log 2>&1
