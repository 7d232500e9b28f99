#!/bin/bash
# Round 6: Gram GEMM units' A loads all at the block start (_ab/early.so, GRAM_A_EARLY 1) vs one per tile
# (_ab/spread.so), each with and without the two-chain T_t units; gradient-only class times at 16 chains, alternating.
O=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/${TAG:-r06i}_ab.txt
D=${GRAFT_REPO_ROOT:-$(pwd)}/_ab
P=profiles/scripts/probes/probe_classes.py
: > $O
for rep in 1 2; do
  for L in spread early; do
    for v in 1 0; do
      VIHMC_LIB=$D/$L.so timeout -k 10 120 python -u $P --chains 16 --iters 20 --grad --opt gram_pair2=$v \
          --tag "$L pair2=$v" >> $O 2>&1 || exit 1
    done
  done
done
grep -v amdgpu.ids $O
