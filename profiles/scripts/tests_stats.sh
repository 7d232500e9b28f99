# GPU tests, then one rocprofv3 kernel-stats pass of a short bench. Usage: bash profiles/scripts/tests_stats.sh <tag>
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/$1; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests.txt 2>&1 && \
cd /tmp && export TMPDIR=/tmp && \
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/s -o s -- python3 $R/bench.py --steps 5 --warmup 1 --cpu-seconds 0 --no-side-legs --ess-steps 0 > $O/s.log 2>&1 && \
python3 $R/profiles/kstats.py $O/s/s_kernel_stats.csv 12 > $O/kstats.txt
