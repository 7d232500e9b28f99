#!/bin/bash
# A/B plan knobs given as environment assignments on the eval probe, one GPU call:
#   bash profiles/ab_env.sh "VIHMC_QSPLIT_A=1" "VIHMC_QSPLIT_A=2 VIHMC_QSPLIT_B=8" ...
set -e
for cfg in "$@"; do
  echo "== $cfg"
  env $cfg timeout -k 10 120 python profiles/scripts/probes/probe_eval.py --chains 16 --iters 30 2>&1 | grep "C="
done
