# Variant library: its GPU parity files first, then the ab_so.sh A/B against the in-tree library.
# Usage: bash profiles/scripts/ab_so_parity.sh <tag> <variant .so>
set -o pipefail
R=$GRAFT_REPO_ROOT; mkdir -p $R/gpurun_out/$1
VIHMC_LIB=$R/_var/$2 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_scale_parity.py tests/test_gpu_api.py -m gpu -x -q --timeout 200 --timeout-method thread > $R/gpurun_out/$1/variant_parity.txt 2>&1 && \
bash $R/profiles/scripts/ab_so.sh $1 $2
