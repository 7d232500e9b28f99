# Input-layer A/B on one box: GPU tests, then bench.py alternating VIHMC_ROWDOT_IN_KF=1 (branch input layer on
# the whole-tile KF = 104 path) and 0 (run-time K for both nets), then rocprofv3 kernel stats of both.
# Usage: bash profiles/scripts/ab_input_layer.sh <tag>
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${1:-r02bg}; mkdir -p $O
B="python3 $R/bench.py --steps 5 --warmup 1 --cpu-seconds 0 --no-side-legs --ess-steps 0"
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests.txt 2>&1 && \
for v in 1 0 1 0; do VIHMC_ROWDOT_IN_KF=$v timeout -k 10 200 python bench.py --steps 20 --warmup 2 --cpu-seconds 0 --no-side-legs --ess-steps 0 >> $O/bench_kf$v.json 2>>$O/bench.err || exit 1; done && \
cd /tmp && export TMPDIR=/tmp && \
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kf1 -o s -- $B > $O/kf1.log 2>&1 && \
VIHMC_ROWDOT_IN_KF=0 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kf0 -o s -- $B > $O/kf0.log 2>&1 && \
cd $R && for v in kf1 kf0; do echo "== $v"; grep -E "k_rowdot" $O/$v/s_kernel_stats.csv | cut -d, -f1-6; done > $O/summary.txt
