#!/bin/bash
# SQ counters of the gradient-only (Gram-form) evaluation at 16 chains, as pmc_sq.sh: one rocprofv3 pass per group
# of 8 SQ counters, each under its own kill timeout. Usage: bash profiles/scripts/pmc_sq_grad.sh <tag>
TAG=${1:-g}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
O=$ROOT/gpurun_out
mkdir -p $O
P="python3 $ROOT/profiles/scripts/probes/probe_classes.py --chains 16 --iters 5 --grad ${OPT:+--opt $OPT}"
G1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE"
G2="SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_UNALIGNED_STALL SQ_ACTIVE_INST_VALU"
cd /tmp && export TMPDIR=/tmp && \
timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv --pmc $G1 -d $O/${TAG}_sq1 -o p -- $P > $O/${TAG}_sq1.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv --pmc $G2 -d $O/${TAG}_sq2 -o p -- $P > $O/${TAG}_sq2.log 2>&1 && \
cd $ROOT && python3 profiles/pmc_kernels.py $O/${TAG}_sq1 > $O/${TAG}_sq.txt && python3 profiles/pmc_kernels.py $O/${TAG}_sq2 >> $O/${TAG}_sq.txt
