cd /tmp && export TMPDIR=/tmp && R=$GRAFT_REPO_ROOT && \
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/g21_base -o s -- python3 $R/profiles/scripts/probes/probe_classes.py --chains 16 --iters 10 --grad > $R/gpurun_out/g21_base.log 2>&1 && \
VIHMC_LIB=$R/_ab/cw4.so timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/g21_cw4 -o s -- python3 $R/profiles/scripts/probes/probe_classes.py --chains 16 --iters 10 --grad > $R/gpurun_out/g21_cw4.log 2>&1
