#!/bin/bash
# Round 6: centred Gram class time after the six-product extension / fp32 dZb epilogue (alternating with the uncentred
# form), then the Gram GPU tests and the good-fit trajectory tests.
O=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out
mkdir -p $O
P=profiles/scripts/probes/probe_classes.py
for rep in 1 2; do
  for v in "gram_center=1" "gram_center=0"; do
    timeout -k 10 120 python -u $P --chains 16 --iters 20 --grad --opt $v --tag "$v" >> $O/${TAG}_ab.txt 2>&1 || exit 1
  done
done
timeout -k 10 500 python -u -m pytest tests/test_gpu_gram.py tests/test_gpu_good_fit.py tests/test_gpu_bench_path.py -q \
    --timeout 200 --timeout-method thread > $O/${TAG}_tests.txt 2>&1
