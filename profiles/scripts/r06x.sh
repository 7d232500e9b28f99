#!/bin/bash
# Round 6: k_gram_a T_b units with B fragments two tiles ahead (_ab/b3.so, GRAM_B3 1) vs one (_ab/b2.so):
# bitwise dumps, gradient-only class times at 16 chains (alternating).
O=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/${TAG:-r06x}
D=${GRAFT_REPO_ROOT:-$(pwd)}/_ab
P=profiles/scripts/probes/probe_classes.py
for L in b2 b3; do
  VIHMC_LIB=$D/$L.so timeout -k 10 100 python -u profiles/scripts/diag/dump_grad.py gpurun_out/dg_$L.npz > /dev/null 2>&1 || exit 1
done
python profiles/scripts/diag/dump_eval.py --compare gpurun_out/dg_b2.npz gpurun_out/dg_b3.npz > ${O}_ab.txt 2>&1
for rep in 1 2 3; do
  for L in b2 b3; do
    VIHMC_LIB=$D/$L.so timeout -k 10 120 python -u $P --chains 16 --iters 20 --grad --tag "$L" >> ${O}_ab.txt 2>&1 || exit 1
  done
done
grep -v amdgpu.ids ${O}_ab.txt
