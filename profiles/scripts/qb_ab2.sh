#!/bin/bash
# Side-B contraction chunks of at least 160 trunk rows (config 4's N = 500 shards: 64 partial slabs instead of 128):
# the one-chain / config-4 GPU tests with the in-tree library, then the legs alternating _ab/base.so / _ab/qb.so.
TAG=${TAG:-r05qb2}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
O=gpurun_out/${TAG}_ab.txt
mkdir -p gpurun_out
export VIHMC_PARITY_LOG=$ROOT/gpurun_out/${TAG}_parity_errors.json
VIHMC_LIB=$ROOT/_ab/qb320.so timeout -k 10 500 python -u -m pytest -x -v --timeout 200 --timeout-method thread -p no:cacheprovider \
    tests/test_gpu_scale_parity.py tests/test_gpu_split_fused.py tests/test_gpu_parity.py tests/test_gpu_sampler.py \
    > gpurun_out/${TAG}_tests.txt 2>&1
rc=$?; tail -3 gpurun_out/${TAG}_tests.txt; [ $rc -eq 0 ] || exit $rc
: > $O
for rep in 1 2 3; do
  for L in qb160 qb320; do
    echo "== $L rep $rep" >> $O
    VIHMC_LIB=$ROOT/_ab/$L.so timeout -k 10 150 python -u profiles/scripts/probes/probe_legs.py --reps 1 >> $O 2>/dev/null || exit 1
  done
done
cat $O
