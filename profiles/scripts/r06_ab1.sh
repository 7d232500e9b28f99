#!/bin/bash
# Round 6: class times of gradient-only evaluations at 16 chains, centred vs uncentred Gram form, tanh_cr on / off
# (alternating, one box), then the driver-like bench line (--steps 20: the sustained leg runs) and rocprofv3 kernel stats.
O=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out
mkdir -p $O
P=profiles/scripts/probes/probe_classes.py
for rep in 1 2; do
  for v in "gram_center=1 tanh_cr=1" "gram_center=0 tanh_cr=1" "gram_center=1 tanh_cr=0"; do
    a=""; for kv in $v; do a="$a --opt $kv"; done
    timeout -k 10 120 python -u $P --chains 16 --iters 20 --grad $a --tag "$v" >> $O/r06_ab1.txt 2>&1 || exit 1
  done
done
timeout -k 10 600 python -u bench.py --steps 20 --cpu-seconds 0 > $O/r06_bench20.json 2> $O/r06_bench20.err || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/r06_stats -o s -- \
    python3 ${GRAFT_REPO_ROOT}/bench.py --steps 40 --warmup 3 --cpu-seconds 0 --no-side-legs --ess-steps 0 \
    > $O/r06_stats.log 2>&1 || exit 1
python3 ${GRAFT_REPO_ROOT}/profiles/kstats.py $(ls $O/r06_stats/*kernel_stats.csv | head -1) 16 > $O/r06_kstats.txt 2>&1
