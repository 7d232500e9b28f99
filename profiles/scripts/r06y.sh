#!/bin/bash
# Round 6: T_b split-K slab count at 16 chains, 8 (the formula, _ab/s0.so) vs 6 / 12 (_ab/s6.so, _ab/s12.so), with the
# centred Gram-t / Gram-b cuts following it: Gram tests on the variants, gradient-only class times (alternating).
O=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/${TAG:-r06y}
D=${GRAFT_REPO_ROOT:-$(pwd)}/_ab
P=profiles/scripts/probes/probe_classes.py
for L in s6 s12; do
  VIHMC_LIB=$D/$L.so timeout -k 10 400 python -u -m pytest tests/test_gpu_gram.py -q -x --timeout 200 \
      --timeout-method thread > ${O}_tests_$L.txt 2>&1 || exit 1
done
: > ${O}_ab.txt
for rep in 1 2 3; do
  for L in s0 s6 s12; do
    VIHMC_LIB=$D/$L.so timeout -k 10 120 python -u $P --chains 16 --iters 20 --grad --tag "$L" >> ${O}_ab.txt 2>&1 || exit 1
  done
done
grep -v amdgpu.ids ${O}_ab.txt
