#!/bin/bash
# Round-6 GPU check of a tree: class A/B of the centred Gram form (gradient-only, 16 chains, alternating), the -m gpu
# suite (VIHMC_PARITY_CALIBRATE=${CAL:-0}), smoke, the driver-like bench line (--steps 20: the sustained leg runs), and
# rocprofv3 kernel stats of a 40-step bench. TAG names the outputs under gpurun_out/. Every GPU step has its own time
# limit; the first failure ends the script.
TAG=${TAG:-r06}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
O=$ROOT/gpurun_out
mkdir -p $O
export VIHMC_PARITY_LOG=$O/${TAG}_parity_errors.json
if [ "${AB:-1}" = 1 ]; then
  for rep in 1 2; do
    for v in "gram_center=1" "gram_center=0"; do
      timeout -k 10 120 python -u profiles/scripts/probes/probe_classes.py --chains 16 --iters 20 --grad --opt $v \
          --tag "$v" >> $O/${TAG}_ab.txt 2>&1 || exit 1
    done
  done
fi
if [ "${TESTS:-1}" = 1 ]; then
  if [ "${CAL:-0}" = 1 ]; then STOP="--maxfail=30"; else STOP="-x"; fi
  VIHMC_PARITY_CALIBRATE=${CAL:-0} timeout -k 10 900 python -u -m pytest tests -m gpu -v $STOP --timeout 300 \
      --timeout-method thread -p no:cacheprovider > $O/${TAG}_tests.txt 2>&1
  rc=$?; echo "tests rc=$rc"; tail -3 $O/${TAG}_tests.txt
  if [ "${CAL:-0}" = 1 ]; then [ $rc -le 1 ] || exit $rc; else [ $rc -eq 0 ] || exit $rc; fi
  timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/${TAG}_smoke.txt 2>&1 || exit 1
fi
[ "${BENCH:-1}" = 1 ] || exit 0
timeout -k 10 600 python -u bench.py --steps 20 > $O/${TAG}_bench.json 2> $O/${TAG}_bench.err; rc=$?; echo "bench rc=$rc"
[ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/${TAG}_stats -o s -- \
    python3 $ROOT/bench.py --steps 40 --warmup 3 --cpu-seconds 0 --no-side-legs --ess-steps 0 \
    > $O/${TAG}_stats.log 2>&1 || exit 1
python3 $ROOT/profiles/kstats.py $(ls $O/${TAG}_stats/*kernel_stats.csv | head -1) 16 > $O/${TAG}_kstats.txt 2>&1
