#!/bin/bash
# Two builds A/B on the bench's timed region (no side legs, no CPU baseline, no ESS phase) and its one-chain legs,
# alternating A, B, A, B. A = _ab/$A.so, B = _ab/$B.so. Output: gpurun_out/${TAG}.txt
TAG=${TAG:-r04bab}; A=${A:-base}; B=${B:-new}
O=gpurun_out/${TAG}.txt
D=${GRAFT_REPO_ROOT:-$(pwd)}/_ab
: > $O
for rep in 1 2; do
  for L in $A $B; do
    echo "== $L rep $rep" >> $O
    VIHMC_LIB=$D/$L.so timeout -k 10 200 python -u bench.py --steps 10 --warmup 2 --cpu-seconds 0 --no-side-legs --ess-steps 0 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('bench', round(d['value'],1), 'ms/step', round(d['ms_per_step'],3), 'sclk', d.get('sclk_mhz'))" >> $O 2>&1 || exit 1
    VIHMC_LIB=$D/$L.so timeout -k 10 150 python -u profiles/scripts/probes/probe_legs.py --reps 1 2>/dev/null >> $O || exit 1
  done
done
cat $O
