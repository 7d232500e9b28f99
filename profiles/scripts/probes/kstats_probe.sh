#!/bin/bash
# rocprofv3 kernel stats of the eval probe at the given chain counts (one GPU call).
# Usage: bash profiles/scripts/probes/kstats_probe.sh <tag> <C> [<C> ...]
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1; shift
cd /tmp && export TMPDIR=/tmp
for C in "$@"; do
  timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $ROOT/gpurun_out/${TAG}_c$C -o s -- \
    python3 $ROOT/profiles/scripts/probes/probe_eval.py --chains $C --iters 20 > $ROOT/gpurun_out/${TAG}_c$C.log 2>&1 || exit $?
done
