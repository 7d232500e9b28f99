#!/bin/bash
# A/B kernel-variant builds (make -C vi-hmc_amd OUT=_var/<name>.so BUILD=build/<name> EXTRA=-D...) on the
# eval probe, one GPU call: bash profiles/ab_variants.sh <name>.so ...
set -e
for f in "$@"; do
  echo "== $f"
  VIHMC_LIB=$GRAFT_REPO_ROOT/_var/$f timeout -k 10 120 python profiles/scripts/probes/probe_eval.py --chains 16 --iters 30 2>&1 | grep "C="
done
