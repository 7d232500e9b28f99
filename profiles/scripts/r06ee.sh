#!/bin/bash
# Round 6: k_gram_b's last round, ablated (VIHMC_DIAG GRB_ABL, switch since removed): 1 = no dZb units, 2 = no T_t
# units past the first two rounds (16 chains), 3 = both; rocprofv3 kernel stats of the gradient-only probe per build.
O=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/${TAG:-r06ee}
D=${GRAFT_REPO_ROOT:-$(pwd)}/_ab
P=profiles/scripts/probes/probe_classes.py
for L in base grb1 grb2 grb3; do
  (cd /tmp && export TMPDIR=/tmp && VIHMC_ALLOW_DIAG=1 VIHMC_LIB=$D/$L.so timeout -k 10 200 rocprofv3 --kernel-trace \
      --stats --output-format csv -d ${O}_prof_$L -o s -- python3 $GRAFT_REPO_ROOT/$P --chains 16 --iters 20 --grad \
      > ${O}_prof_$L.log 2>&1) || exit 1
  echo "== $L" >> ${O}_kstats.txt
  python3 profiles/kstats.py $(ls ${O}_prof_$L/*kernel_stats.csv | head -1) 16 | grep gram >> ${O}_kstats.txt 2>&1
done
cat ${O}_kstats.txt
