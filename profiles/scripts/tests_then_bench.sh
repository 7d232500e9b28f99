#!/bin/bash
# One GPU call: selected GPU tests, then the default bench line. Usage: tests_then_bench.sh <tag> <pytest args...>
set -o pipefail
TAG=$1
shift
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -m gpu -x -v -s --timeout 300 --timeout-method thread "$@" \
    > gpurun_out/${TAG}_tests.txt 2>&1 && \
timeout -k 10 400 python bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err
