#!/bin/bash
# Round 6: the centred form's Gram-t units split GRAM_T_SPLIT = 1 / 2 / 4 times per T_b slab (_ab/ts{1,2,4}.so):
# the Gram tests on each variant (the split changes the Gt / Ht slab sums' order), class times at 16 chains
# (alternating), rocprofv3 kernel stats.
O=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/${TAG:-r06p}
D=${GRAFT_REPO_ROOT:-$(pwd)}/_ab
P=profiles/scripts/probes/probe_classes.py
for L in ts2 ts4; do
  VIHMC_LIB=$D/$L.so timeout -k 10 400 python -u -m pytest tests/test_gpu_gram.py tests/test_gpu_good_fit.py -q -x \
      --timeout 200 --timeout-method thread > ${O}_tests_$L.txt 2>&1 || exit 1
done
: > ${O}_ab.txt
for rep in 1 2 3; do
  for L in ts1 ts2 ts4; do
    VIHMC_LIB=$D/$L.so timeout -k 10 120 python -u $P --chains 16 --iters 20 --grad --tag "$L" >> ${O}_ab.txt 2>&1 || exit 1
  done
done
for L in ts1 ts2 ts4; do
  (cd /tmp && export TMPDIR=/tmp && VIHMC_LIB=$D/$L.so timeout -k 10 200 rocprofv3 --kernel-trace --stats \
      --output-format csv -d ${O}_prof_$L -o s -- python3 $GRAFT_REPO_ROOT/$P --chains 16 --iters 20 --grad \
      > ${O}_prof_$L.log 2>&1) || exit 1
  python3 profiles/kstats.py $(ls ${O}_prof_$L/*kernel_stats.csv | head -1) 16 > ${O}_kstats_$L.txt 2>&1
done
grep -v amdgpu.ids ${O}_ab.txt
