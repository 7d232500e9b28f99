#!/bin/bash
# FETCH_SIZE of the Gram kernels, in-tree library vs _ab/<v>.so (gradient-only probe, 16 chains), one PMC pass each.
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}; TAG=$1; V=$2
cd /tmp && export TMPDIR=/tmp && \
timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv --pmc FETCH_SIZE -d $ROOT/gpurun_out/${TAG}_new -o p -- python3 $ROOT/profiles/scripts/probes/probe_classes.py --chains 16 --iters 5 --grad > $ROOT/gpurun_out/${TAG}_new.log 2>&1 && \
VIHMC_LIB=$ROOT/_ab/$V.so timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv --pmc FETCH_SIZE -d $ROOT/gpurun_out/${TAG}_$V -o p -- python3 $ROOT/profiles/scripts/probes/probe_classes.py --chains 16 --iters 5 --grad > $ROOT/gpurun_out/${TAG}_$V.log 2>&1
