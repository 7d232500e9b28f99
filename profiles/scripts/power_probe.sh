#!/bin/bash
# Board power and clocks while the C=16 evaluation probe runs (rocm-smi sampled in the background).
# Usage: bash profiles/scripts/power_probe.sh <tag>
TAG=${1:-r03}
mkdir -p gpurun_out
( for i in $(seq 1 40); do rocm-smi --showpower --showclocks --showtemp 2>/dev/null | grep -E "Power|sclk|fclk|mclk|Temp" ; echo ---; sleep 0.25; done ) > gpurun_out/${TAG}_power.txt 2>&1 &
SMI=$!
timeout -k 10 120 python profiles/scripts/probes/probe_classes.py --chains 16 --iters 400 ${GRAD:+--grad} > gpurun_out/${TAG}_power_probe.txt 2>&1
RC=$?
wait $SMI
exit $RC
