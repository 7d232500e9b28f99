#!/bin/bash
# Round 6: k_gram_a unit order, Gram units first (shipped, _ab/gfirst.so) vs T_b units first (_ab/tfirst.so), with the
# round-6 unit cuts; gradient-only class times at 16 chains (alternating) and rocprofv3 kernel stats.
O=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/${TAG:-r06u}
D=${GRAFT_REPO_ROOT:-$(pwd)}/_ab
P=profiles/scripts/probes/probe_classes.py
: > ${O}_ab.txt
for rep in 1 2 3; do
  for L in gfirst tfirst; do
    VIHMC_LIB=$D/$L.so timeout -k 10 120 python -u $P --chains 16 --iters 20 --grad --tag "$L" >> ${O}_ab.txt 2>&1 || exit 1
  done
done
grep -v amdgpu.ids ${O}_ab.txt
