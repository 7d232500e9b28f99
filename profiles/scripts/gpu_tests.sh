#!/bin/bash
# One GPU call: selected GPU tests. Usage: bash profiles/scripts/gpu_tests.sh <tag> <pytest args...>
set -o pipefail
TAG=$1
shift
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest -m gpu -x -v -s --timeout 300 --timeout-method thread "$@" > gpurun_out/${TAG}_tests.txt 2>&1
