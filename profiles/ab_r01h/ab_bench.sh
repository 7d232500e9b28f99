#!/bin/bash
set -e
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out
B="python3 $R/bench.py --steps 60 --warmup 5 --cpu-seconds 0 --ess-steps 0"
for i in 1 2 3; do
  timeout -k 10 120 $B > $O/abb_new_$i.json 2>/dev/null
  VIHMC_LIB=$R/_var/old2.so timeout -k 10 120 $B > $O/abb_old_$i.json 2>/dev/null
done
