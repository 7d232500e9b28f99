#!/bin/bash
# Round 6: matrix-pipe priority of the Gram GEMM units' wave pairs (GRAM_PRIO 0 / 1 / 2: _ab/prio{0,1,2}.so):
# bitwise dumps (priority changes timing only), gradient-only class times at 16 chains (alternating).
O=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/${TAG:-r06w}
D=${GRAFT_REPO_ROOT:-$(pwd)}/_ab
P=profiles/scripts/probes/probe_classes.py
for L in prio0 prio1 prio2; do
  VIHMC_LIB=$D/$L.so timeout -k 10 100 python -u profiles/scripts/diag/dump_grad.py gpurun_out/dg_$L.npz > /dev/null 2>&1 || exit 1
done
python profiles/scripts/diag/dump_eval.py --compare gpurun_out/dg_prio0.npz gpurun_out/dg_prio1.npz > ${O}_ab.txt 2>&1
python profiles/scripts/diag/dump_eval.py --compare gpurun_out/dg_prio0.npz gpurun_out/dg_prio2.npz >> ${O}_ab.txt 2>&1
for rep in 1 2 3; do
  for L in prio0 prio1 prio2; do
    VIHMC_LIB=$D/$L.so timeout -k 10 120 python -u $P --chains 16 --iters 20 --grad --tag "$L" >> ${O}_ab.txt 2>&1 || exit 1
  done
done
grep -v amdgpu.ids ${O}_ab.txt
