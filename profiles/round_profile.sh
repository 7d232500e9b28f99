#!/bin/bash
# Round evidence on the GPU box: default bench line, its rocprofv3 kernel stats, and the two PMC passes that
# give every kernel's HBM traffic per launch (profiles/traffic.json format). Each GPU step has its own time
# limit and the steps are chained with &&: a failure ends the call.
# Usage: bash profiles/round_profile.sh <tag>
TAG=${1:-r02}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
O=$ROOT/gpurun_out
mkdir -p $O
B="python3 $ROOT/bench.py --steps 5 --warmup 1 --cpu-seconds 0 --no-side-legs"
timeout -k 10 600 python3 $ROOT/bench.py > $O/${TAG}_bench.json 2> $O/${TAG}_bench.err && \
cd /tmp && export TMPDIR=/tmp && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/${TAG}_stats -o s -- $B \
    > $O/${TAG}_stats.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv --pmc FETCH_SIZE -d $O/${TAG}_fetch -o p -- \
    $B --ess-steps 0 > $O/${TAG}_fetch.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv --pmc WRITE_SIZE -d $O/${TAG}_write -o p -- \
    $B --ess-steps 0 > $O/${TAG}_write.log 2>&1 && \
cd $ROOT && \
python3 profiles/traffic_from_pmc.py $O/${TAG}_fetch $O/${TAG}_write $O/${TAG}_traffic.json 16 "${TAG} bench PMC passes" \
    > $O/${TAG}_traffic.log 2>&1 && \
python3 profiles/kstats.py $(ls $O/${TAG}_stats/*kernel_stats.csv | head -1) 30 > $O/${TAG}_kstats.txt 2>&1
