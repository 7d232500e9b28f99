#!/bin/bash
# Round 6: k_gram_b's main loop two blocks per barrier (_ab/bpair.so, GRB_PAIR 1) vs one (_ab/base.so): the Gram GPU
# tests on the variant, bitwise dumps of both, gradient-only class times at 16 chains (alternating).
O=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/${TAG:-r06m}
D=${GRAFT_REPO_ROOT:-$(pwd)}/_ab
P=profiles/scripts/probes/probe_classes.py
VIHMC_LIB=$D/bpair.so timeout -k 10 400 python -u -m pytest tests/test_gpu_gram.py tests/test_gpu_good_fit.py -q \
    --timeout 200 --timeout-method thread > ${O}_tests.txt 2>&1 || exit 1
for L in base bpair; do
  VIHMC_LIB=$D/$L.so timeout -k 10 100 python -u profiles/scripts/diag/dump_eval.py gpurun_out/dump_$L.npz > /dev/null 2>&1 || exit 1
done
python profiles/scripts/diag/dump_eval.py --compare gpurun_out/dump_base.npz gpurun_out/dump_bpair.npz > ${O}_ab.txt 2>&1
for rep in 1 2 3; do
  for L in base bpair; do
    VIHMC_LIB=$D/$L.so timeout -k 10 120 python -u $P --chains 16 --iters 20 --grad --tag "$L" >> ${O}_ab.txt 2>&1 || exit 1
  done
done
grep -v amdgpu.ids ${O}_ab.txt
