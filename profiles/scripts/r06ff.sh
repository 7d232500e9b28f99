#!/bin/bash
# Round 6: dZb epilogue units of DZB_RS = 1 / 2 / 4 32-row groups sharing one Gt / Ht staging (_ab/rs{1,2,4}.so):
# bitwise dumps, the dZb units alone (gram_pair2 = 2 leaves k_gram_b<1> only them) under rocprofv3, gradient-only
# class times at 16 chains (alternating).
O=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/${TAG:-r06ff}
D=${GRAFT_REPO_ROOT:-$(pwd)}/_ab
P=profiles/scripts/probes/probe_classes.py
for L in rs1 rs2 rs4; do
  VIHMC_LIB=$D/$L.so timeout -k 10 100 python -u profiles/scripts/diag/dump_grad.py gpurun_out/dg_$L.npz > /dev/null 2>&1 || exit 1
done
python profiles/scripts/diag/dump_eval.py --compare gpurun_out/dg_rs1.npz gpurun_out/dg_rs2.npz > ${O}_ab.txt 2>&1
python profiles/scripts/diag/dump_eval.py --compare gpurun_out/dg_rs1.npz gpurun_out/dg_rs4.npz >> ${O}_ab.txt 2>&1
for L in rs1 rs2 rs4; do
  (cd /tmp && export TMPDIR=/tmp && VIHMC_LIB=$D/$L.so timeout -k 10 200 rocprofv3 --kernel-trace --stats \
      --output-format csv -d ${O}_prof_$L -o s -- python3 $GRAFT_REPO_ROOT/$P --chains 16 --iters 20 --grad \
      --opt gram_pair2=2 > ${O}_prof_$L.log 2>&1) || exit 1
  echo "== $L (gram_pair2 = 2: k_gram_b<1> = the dZb units)" >> ${O}_ab.txt
  python3 profiles/kstats.py $(ls ${O}_prof_$L/*kernel_stats.csv | head -1) 16 | grep gram_b >> ${O}_ab.txt 2>&1
done
for rep in 1 2 3; do
  for L in rs1 rs2 rs4; do
    VIHMC_LIB=$D/$L.so timeout -k 10 120 python -u $P --chains 16 --iters 20 --grad --tag "$L" >> ${O}_ab.txt 2>&1 || exit 1
  done
done
grep -v amdgpu.ids ${O}_ab.txt
