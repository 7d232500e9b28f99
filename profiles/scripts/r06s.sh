#!/bin/bash
# Round 6: GRAM_T_SPLIT 3 (_ab/t3.so) vs 2 (_ab/t2.so), the Gram-b units cut alike: Gram tests on the variant, class
# times at 16 chains (alternating).
O=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/${TAG:-r06s}
D=${GRAFT_REPO_ROOT:-$(pwd)}/_ab
P=profiles/scripts/probes/probe_classes.py
VIHMC_LIB=$D/t3.so timeout -k 10 400 python -u -m pytest tests/test_gpu_gram.py -q -x --timeout 200 \
    --timeout-method thread > ${O}_tests.txt 2>&1 || exit 1
: > ${O}_ab.txt
for rep in 1 2 3; do
  for L in t2 t3; do
    VIHMC_LIB=$D/$L.so timeout -k 10 120 python -u $P --chains 16 --iters 20 --grad --tag "$L" >> ${O}_ab.txt 2>&1 || exit 1
  done
done
grep -v amdgpu.ids ${O}_ab.txt
