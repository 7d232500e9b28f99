# In-tree library vs one variant build on one box: GPU tests on the in-tree library, bench.py alternating the two
# (VIHMC_LIB), then rocprofv3 kernel stats of a short bench for each.
# Usage: bash profiles/scripts/ab_so.sh <tag> <variant .so under _var/>
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/$1; V=$R/_var/$2; mkdir -p $O
B="python3 $R/bench.py --steps 5 --warmup 1 --cpu-seconds 0 --no-side-legs --ess-steps 0"
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests.txt 2>&1 && \
for i in 1 2; do \
  timeout -k 10 200 python bench.py --steps 20 --warmup 2 --cpu-seconds 0 --no-side-legs --ess-steps 0 >> $O/bench_new.json 2>>$O/bench.err && \
  VIHMC_LIB=$V timeout -k 10 200 python bench.py --steps 20 --warmup 2 --cpu-seconds 0 --no-side-legs --ess-steps 0 >> $O/bench_old.json 2>>$O/bench.err || exit 1; done && \
cd /tmp && export TMPDIR=/tmp && \
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/new -o s -- $B > $O/new.log 2>&1 && \
VIHMC_LIB=$V timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/old -o s -- $B > $O/old.log 2>&1 && \
cd $R && for v in new old; do echo "== $v"; python3 profiles/kstats.py $O/$v/s_kernel_stats.csv 10; done > $O/summary.txt
