#!/bin/bash
# Reducer workgroups: tests (in-tree library), legs alternating base / red / idle (reducers publish-only, no tasks:
# the compute workgroups' own time), and kernel traces of red and idle.
TAG=${TAG:-r05cr3}
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
  for L in base red idle; do
    echo "== $L rep $rep" >> $O
    VIHMC_LIB=$ROOT/_ab/$L.so timeout -k 10 150 python -u profiles/scripts/probes/probe_legs.py --reps 1 >> $O 2>/dev/null || exit 1
  done
done
cat $O
cd /tmp && export TMPDIR=/tmp
for L in red idle; do
  VIHMC_LIB=$ROOT/_ab/$L.so timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d $ROOT/gpurun_out/${TAG}_kt_$L -o t -- \
      python3 $ROOT/profiles/scripts/probes/probe_legs.py --reps 1 > $ROOT/gpurun_out/${TAG}_kt_$L.log 2>&1 || exit 1
  python3 $ROOT/profiles/scripts/diag/trace_summary.py $(ls $ROOT/gpurun_out/${TAG}_kt_$L/*kernel_trace.csv | head -1) > $ROOT/gpurun_out/${TAG}_trace_$L.txt 2>&1
  echo "== trace $L"; head -8 $ROOT/gpurun_out/${TAG}_trace_$L.txt
done
