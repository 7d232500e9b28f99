#!/bin/bash
# PMC passes (one counter group per rocprofv3 run, --kernel-trace only, never combined with sys/runtime
# traces) over a short C=16 eval probe. Usage (GPU box): bash profiles/pmc_passes.sh <outdir-name>
# Outputs under gpurun_out/<name>_{a..e}/; summarise with: python profiles/pmc_summary.py gpurun_out/<name>
set -e
NAME=${1:-pmc}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp && export TMPDIR=/tmp
P="python3 $ROOT/profiles/scripts/probes/probe_eval.py --chains 16 --iters 3"
run() {
    local tag=$1; shift
    timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv --pmc "$@" -d "$ROOT/gpurun_out/${NAME}_$tag" -o p -- $P \
        > "$ROOT/gpurun_out/${NAME}_$tag.log" 2>&1
}
run a SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES GRBM_GUI_ACTIVE
run b SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_VALU_MFMA_BUSY_CYCLES SQ_VALU_MFMA_COEXEC_CYCLES SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE
run c SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LEVEL_WAVES
run d SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE FETCH_SIZE
run e WRITE_SIZE
