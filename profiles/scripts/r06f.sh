#!/bin/bash
O=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out
mkdir -p $O
timeout -k 10 300 python -u profiles/scripts/diag/resid_parts_err.py 1e-2 1e-3 1e-5 > $O/r06f_resid_parts.txt 2>&1 || exit 1
timeout -k 10 120 python -u profiles/scripts/probes/probe_classes.py --chains 16 --iters 20 --tag full16 > $O/r06f_classes.txt 2>&1 || exit 1
timeout -k 10 120 python -u profiles/scripts/probes/probe_classes.py --chains 1 --iters 40 --tag full1 >> $O/r06f_classes.txt 2>&1 || exit 1
timeout -k 10 600 python -u -m pytest tests/test_gpu_gram.py -q --timeout 200 --timeout-method thread -k precision_vs_fit > $O/r06f_tests.txt 2>&1
