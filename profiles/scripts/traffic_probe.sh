#!/bin/bash
# FETCH_SIZE / WRITE_SIZE per kernel of the C=16 evaluation probe (two PMC passes). Usage: traffic_probe.sh <tag>
TAG=${1:-r03}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
O=$ROOT/gpurun_out
mkdir -p $O
P="python3 $ROOT/profiles/scripts/probes/probe_classes.py --chains 16 --iters 5 ${GRAD:+--grad} ${OPT:+--opt $OPT}"
cd /tmp && export TMPDIR=/tmp && \
timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv --pmc FETCH_SIZE -d $O/${TAG}_fetch -o p -- $P > $O/${TAG}_fetch.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv --pmc WRITE_SIZE -d $O/${TAG}_write -o p -- $P > $O/${TAG}_write.log 2>&1 && \
cd $ROOT && python3 profiles/traffic_from_pmc.py $O/${TAG}_fetch $O/${TAG}_write $O/${TAG}_traffic.json 16 "${TAG} probe PMC passes" > $O/${TAG}_traffic.log 2>&1
