#!/bin/bash
# Round 6: forward ablations at 16 chains (VIHMC_DIAG FWD_ABL: 1 = no h stores, 2 = tanh -> identity) against the
# shipped build, gradient-only evaluations, alternating. Timing only (the ablations change results).
O=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/${TAG:-r06j}_ab.txt
D=${GRAFT_REPO_ROOT:-$(pwd)}/_ab
P=profiles/scripts/probes/probe_classes.py
: > $O
for rep in 1 2; do
  for L in base fabl1 fabl2; do
    VIHMC_ALLOW_DIAG=1 VIHMC_LIB=$D/$L.so timeout -k 10 120 python -u $P --chains 16 --iters 20 --grad --tag "$L" >> $O 2>&1 || exit 1
  done
done
grep -v amdgpu.ids $O
