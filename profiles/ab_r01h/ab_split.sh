#!/bin/bash
set -e
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > $O/split_parity.log 2>&1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/split_new -o s -- python3 $R/profiles/scripts/probes/probe_eval.py --chains 16 --iters 30 > $O/split_new.log 2>&1
VIHMC_LIB=$R/_var/split4.so timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/split_old -o s -- python3 $R/profiles/scripts/probes/probe_eval.py --chains 16 --iters 30 > $O/split_old.log 2>&1
