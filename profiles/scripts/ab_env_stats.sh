# Run-time knob A/B with kernel statistics: GPU tests once, then per setting one rocprofv3 --kernel-trace --stats
# pass over a short bench, summarised by profiles/kstats.py. Usage: bash profiles/scripts/ab_env_stats.sh <tag> "ENV=a" ...
set -o pipefail
R=$GRAFT_REPO_ROOT; TAG=$1; shift; O=$R/gpurun_out/$TAG; mkdir -p $O
B="python3 $R/bench.py --steps 5 --warmup 1 --cpu-seconds 0 --no-side-legs --ess-steps 0"
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests.txt 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp
i=0
for kv in "$@"; do
  i=$((i+1))
  env $kv timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/s$i -o s -- $B > $O/s$i.log 2>&1 || exit 1
  (echo "== $kv"; python3 $R/profiles/kstats.py $O/s$i/s_kernel_stats.csv 8) >> $O/summary.txt || exit 1
done
