#!/bin/bash
# Reducer workgroups with the last layers' reduce left to a k_reduce launch (plan option chain_red_tail = T):
# tests (in-tree library), then the one-chain legs alternating base and the T variants (_ab/t$T.so).
TAG=${TAG:-r05ct}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
O=gpurun_out/${TAG}_ab.txt
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread -p no:cacheprovider \
    "tests/test_gpu_parity.py::test_single_chain_kernels_bitwise_equal_batched_kernels" \
    tests/test_gpu_split_fused.py tests/test_gpu_scale_parity.py tests/test_gpu_sampler.py \
    > gpurun_out/${TAG}_tests.txt 2>&1
rc=$?; tail -3 gpurun_out/${TAG}_tests.txt; [ $rc -eq 0 ] || exit $rc
: > $O
for rep in 1 2; do
  for L in ${LIBS:-base t0 t2 t3 t4}; do
    echo "== $L rep $rep" >> $O
    VIHMC_LIB=$ROOT/_ab/$L.so timeout -k 10 150 python -u profiles/scripts/probes/probe_legs.py --reps 1 >> $O 2>/dev/null || exit 1
  done
done
cat $O
