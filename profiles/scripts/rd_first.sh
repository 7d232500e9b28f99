# Input-layer launch with the branch workgroups only (_var/rdfirst.so, RD_ONLY_FIRST=1 timing build) vs both nets:
# rocprofv3 kernel stats of a short bench each. Usage: bash profiles/scripts/rd_first.sh <tag>
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/$1; mkdir -p $O
B="python3 $R/bench.py --steps 3 --warmup 1 --cpu-seconds 0 --no-side-legs --ess-steps 0"
cd /tmp && export TMPDIR=/tmp && \
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/both -o s -- $B > $O/both.log 2>&1 && \
VIHMC_ALLOW_DIAG=1 VIHMC_LIB=$R/_var/rdfirst.so timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/first -o s -- $B > $O/first.log 2>&1 && \
cd $R && for v in both first; do echo "== $v"; grep -E "k_rowdot" $O/$v/s_kernel_stats.csv | cut -d, -f1-4; done > $O/summary.txt
