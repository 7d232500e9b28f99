#!/bin/bash
# rocprofv3 kernel stats of probe_crossover.py at one chain count (one GPU call); prints the top kernels.
# Usage: bash profiles/scripts/probes/kstats_cross.sh <tag> <C> [<rows>]
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1; C=$2; ROWS=${3:-1000}
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $ROOT/gpurun_out/${TAG} -o s -- \
  python3 $ROOT/profiles/scripts/probes/probe_crossover.py --chains $C --rows $ROWS --iters 40 --reps 1 > $ROOT/gpurun_out/${TAG}.log 2>&1 || exit $?
python3 $ROOT/profiles/kstats.py $ROOT/gpurun_out/${TAG}/s_kernel_stats.csv > $ROOT/gpurun_out/${TAG}_kstats.txt 2>&1
cat $ROOT/gpurun_out/${TAG}_kstats.txt | head -30
