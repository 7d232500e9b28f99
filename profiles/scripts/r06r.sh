#!/bin/bash
# Round 6: Gram-b units cut like the centred Gram-t units (_ab/sb2.so: two slabs of 20 branch blocks at 16 chains) vs
# one slab of 32 (_ab/sb1.so): Gram tests on the variant, class times at 16 chains (alternating).
O=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/${TAG:-r06r}
D=${GRAFT_REPO_ROOT:-$(pwd)}/_ab
P=profiles/scripts/probes/probe_classes.py
VIHMC_LIB=$D/sb2.so timeout -k 10 400 python -u -m pytest tests/test_gpu_gram.py -q -x --timeout 200 \
    --timeout-method thread > ${O}_tests.txt 2>&1 || exit 1
: > ${O}_ab.txt
for rep in 1 2 3; do
  for L in sb1 sb2; do
    VIHMC_LIB=$D/$L.so timeout -k 10 120 python -u $P --chains 16 --iters 20 --grad --tag "$L" >> ${O}_ab.txt 2>&1 || exit 1
  done
done
grep -v amdgpu.ids ${O}_ab.txt
