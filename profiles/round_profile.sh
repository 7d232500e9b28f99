#!/bin/bash
# Round-end evidence on the GPU box: default bench line, its rocprofv3 kernel stats, and the two PMC
# passes that give the roofline kernel's HBM traffic. Usage: bash profiles/round_profile.sh <tag>
set -e
TAG=${1:-r01}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
O=$ROOT/gpurun_out
timeout -k 10 600 python3 $ROOT/bench.py > $O/${TAG}_bench.json 2> $O/${TAG}_bench.err
cd /tmp && export TMPDIR=/tmp
B="python3 $ROOT/bench.py --steps 5 --warmup 1 --cpu-seconds 0"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/${TAG}_stats -o s -- $B > $O/${TAG}_stats.log 2>&1
# PMC passes without the ESS phase: its device->host sample copies crashed inside torch's copy kernel
# under the PMC tool (r01d); the side-A contraction launches are the same either way.
B="$B --ess-steps 0"
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv --pmc FETCH_SIZE -d $O/${TAG}_fetch -o p -- $B > $O/${TAG}_fetch.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv --pmc WRITE_SIZE -d $O/${TAG}_write -o p -- $B > $O/${TAG}_write.log 2>&1
python3 $ROOT/profiles/traffic_from_pmc.py $O/${TAG}_fetch $O/${TAG}_write $O/${TAG}_traffic.json 16 > $O/${TAG}_traffic.log 2>&1
cd $ROOT && python3 profiles/kstats.py $(ls $O/${TAG}_stats/*kernel_stats.csv | head -1) 30 > $O/${TAG}_kstats.txt 2>&1 || true
