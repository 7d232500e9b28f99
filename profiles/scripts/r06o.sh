#!/bin/bash
# Round 6: the centred dZb epilogue's products on the exact f32 MFMA (_ab/dzbm.so) vs the VALU fmaf loop
# (_ab/base.so): bitwise dumps of gradient-only and log-prob evaluations, the Gram tests on the variant, the dZb units
# alone (gram_pair2 = 2 leaves k_gram_b<1> only them) under rocprofv3, class times at 16 chains.
O=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/${TAG:-r06o}
D=${GRAFT_REPO_ROOT:-$(pwd)}/_ab
P=profiles/scripts/probes/probe_classes.py
for L in base dzbm; do
  VIHMC_LIB=$D/$L.so timeout -k 10 100 python -u profiles/scripts/diag/dump_grad.py gpurun_out/dg_$L.npz > /dev/null 2>&1 || exit 1
  VIHMC_LIB=$D/$L.so timeout -k 10 100 python -u profiles/scripts/diag/dump_eval.py gpurun_out/de_$L.npz > /dev/null 2>&1 || exit 1
done
python profiles/scripts/diag/dump_eval.py --compare gpurun_out/dg_base.npz gpurun_out/dg_dzbm.npz > ${O}_ab.txt 2>&1
python profiles/scripts/diag/dump_eval.py --compare gpurun_out/de_base.npz gpurun_out/de_dzbm.npz >> ${O}_ab.txt 2>&1
VIHMC_LIB=$D/dzbm.so timeout -k 10 400 python -u -m pytest tests/test_gpu_gram.py tests/test_gpu_good_fit.py -q \
    --timeout 200 --timeout-method thread > ${O}_tests.txt 2>&1 || exit 1
for L in base dzbm; do
  (cd /tmp && export TMPDIR=/tmp && VIHMC_LIB=$D/$L.so timeout -k 10 200 rocprofv3 --kernel-trace --stats \
      --output-format csv -d ${O}_prof_$L -o s -- python3 $GRAFT_REPO_ROOT/$P --chains 16 --iters 20 --grad \
      --opt gram_pair2=2 > ${O}_prof_$L.log 2>&1) || exit 1
  python3 profiles/kstats.py $(ls ${O}_prof_$L/*kernel_stats.csv | head -1) 16 > ${O}_kstats_$L.txt 2>&1
done
for rep in 1 2 3; do
  for L in base dzbm; do
    VIHMC_LIB=$D/$L.so timeout -k 10 120 python -u $P --chains 16 --iters 20 --grad --tag "$L" >> ${O}_ab.txt 2>&1 || exit 1
  done
done
grep -v amdgpu.ids ${O}_ab.txt
