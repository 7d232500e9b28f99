# Input-layer kernel, per part: rocprofv3 kernel stats of a short bench for the in-tree library (both nets),
# _var/in1.so (branch workgroups only) and _var/in2.so (trunk only) -- IN_ONLY timing builds -- and the
# k_rowdot2 form (VIHMC_INPUT_VALU=0). Usage: bash profiles/scripts/ab_input_parts.sh <tag>
set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${1:-r02be}; mkdir -p $O
B="python3 $R/bench.py --steps 3 --warmup 1 --cpu-seconds 0 --no-side-legs --ess-steps 0"
cd /tmp && export TMPDIR=/tmp && \
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/def -o s -- $B > $O/def.log 2>&1 && \
VIHMC_ALLOW_DIAG=1 VIHMC_LIB=$R/_var/in1.so timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/in1 -o s -- $B > $O/in1.log 2>&1 && \
VIHMC_ALLOW_DIAG=1 VIHMC_LIB=$R/_var/in2.so timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/in2 -o s -- $B > $O/in2.log 2>&1 && \
VIHMC_INPUT_VALU=0 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/rowdot -o s -- $B > $O/rowdot.log 2>&1 && \
cd $R && for v in def in1 in2 rowdot; do echo "== $v"; grep -E "k_input_layer|k_rowdot2" $O/$v/s_kernel_stats.csv | cut -d, -f1-6; done > $O/summary.txt
