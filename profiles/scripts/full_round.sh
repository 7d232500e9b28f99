#!/bin/bash
# One GPU call: every GPU test, smoke(), then profiles/round_profile.sh (bench line + rocprofv3 stats + PMC
# traffic). Usage: bash profiles/scripts/full_round.sh <tag>
set -o pipefail
TAG=${1:-r02}
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
    > gpurun_out/${TAG}_gpu_tests.txt 2>&1 && \
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.txt 2>&1 && \
bash profiles/round_profile.sh $TAG
