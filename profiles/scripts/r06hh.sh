#!/bin/bash
# Round 6: k_gram_b unit order, dZb units last (shipped, _ab/dlast.so) vs first (_ab/dfirst.so), with the
# round-6 unit cuts; gradient-only class times at 16 chains (alternating) and rocprofv3 kernel stats.
O=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/${TAG:-r06hh}
D=${GRAFT_REPO_ROOT:-$(pwd)}/_ab
P=profiles/scripts/probes/probe_classes.py
: > ${O}_ab.txt
for rep in 1 2 3; do
  for L in dlast dfirst; do
    VIHMC_LIB=$D/$L.so timeout -k 10 120 python -u $P --chains 16 --iters 20 --grad --tag "$L" >> ${O}_ab.txt 2>&1 || exit 1
  done
done
grep -v amdgpu.ids ${O}_ab.txt
