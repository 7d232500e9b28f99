#!/bin/bash
# Round 6: Gram ablations at 16 chains (VIHMC_DIAG GR_ABL: 1 = A loads from block 0 only, 2 = no block DMA, 3 = both)
# against the shipped build, gradient-only class times, alternating. Timing only (the ablations change results).
O=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/${TAG:-r06l}_ab.txt
D=${GRAFT_REPO_ROOT:-$(pwd)}/_ab
P=profiles/scripts/probes/probe_classes.py
: > $O
for rep in 1 2; do
  for L in base gabl1 gabl2 gabl3; do
    VIHMC_ALLOW_DIAG=1 VIHMC_LIB=$D/$L.so timeout -k 10 120 python -u $P --chains 16 --iters 20 --grad --tag "$L" >> $O 2>&1 || exit 1
  done
done
grep -v amdgpu.ids $O
