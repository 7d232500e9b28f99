#!/bin/bash
# Probe + kernel trace at C=1 and C=16, then SQ counters at C=16. Usage: baseline_c1_c16.sh <tag>
TAG=${1:-r03c}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd $ROOT
bash profiles/scripts/ktrace_c.sh ${TAG}_c1 1 && \
bash profiles/scripts/ktrace_c.sh ${TAG}_c16 16 && \
bash profiles/scripts/pmc_sq.sh ${TAG} && \
cd $ROOT && python3 profiles/ktrace_eval.py gpurun_out/${TAG}_c1_kt > gpurun_out/${TAG}_c1_eval.txt && \
python3 profiles/ktrace_eval.py gpurun_out/${TAG}_c16_kt > gpurun_out/${TAG}_c16_eval.txt
