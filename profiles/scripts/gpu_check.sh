#!/bin/bash
# One GPU call: parity tests, smoke, default bench line. Usage: bash profiles/scripts/gpu_check.sh <tag> [pytest args]
set -o pipefail
TAG=${1:-r02}
shift
O=gpurun_out
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 180 --timeout-method thread "$@" > $O/${TAG}_gpu_tests.txt 2>&1 && \
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > $O/${TAG}_smoke.txt 2>&1 && \
timeout -k 10 400 python bench.py > $O/${TAG}_bench.json 2> $O/${TAG}_bench.err
