#!/bin/bash
# Two builds A/B (round 4): bitwise dumps (dump_eval.py), gradient-only and full-evaluation class timings at 16
# chains, the one-chain crossover, alternating A, B, A, B. A = _ab/$A.so, B = _ab/$B.so.
# Output: gpurun_out/${TAG}.txt
TAG=${TAG:-r04ab}; A=${A:-base}; B=${B:-noslp}
O=gpurun_out/${TAG}.txt
D=${GRAFT_REPO_ROOT:-$(pwd)}/_ab
: > $O
for L in $A $B; do
  VIHMC_LIB=$D/$L.so timeout -k 10 100 python -u profiles/scripts/diag/dump_eval.py gpurun_out/dump_$L.npz >> $O 2>&1 || exit 1
done
python profiles/scripts/diag/dump_eval.py --compare gpurun_out/dump_$A.npz gpurun_out/dump_$B.npz >> $O 2>&1
for rep in 1 2; do
  for L in $A $B; do
    echo "== $L rep $rep" >> $O
    VIHMC_LIB=$D/$L.so timeout -k 10 100 python -u profiles/scripts/probes/probe_classes.py --chains 16 --iters 30 --grad >> $O 2>&1 || exit 1
    VIHMC_LIB=$D/$L.so timeout -k 10 100 python -u profiles/scripts/probes/probe_classes.py --chains 16 --iters 30 >> $O 2>&1 || exit 1
    VIHMC_LIB=$D/$L.so timeout -k 10 200 python -u profiles/scripts/probes/probe_crossover.py --chains 1 --rows 1000 500 --reps 1 >> $O 2>&1 || exit 1
  done
done
grep -v amdgpu.ids $O
