# One-chain A/B of a variant library: GPU tests on the in-tree library, then the C = 1 probe + kernel trace for the
# in-tree library and for _var/<variant>. Usage: bash profiles/scripts/ab_c1_so.sh <tag> <variant .so>
set -o pipefail
R=$GRAFT_REPO_ROOT; mkdir -p $R/gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $R/gpurun_out/$1_gpu_tests.txt 2>&1 && \
bash $R/profiles/scripts/ktrace_c.sh $1_new 1 && \
VIHMC_LIB=$R/_var/$2 bash $R/profiles/scripts/ktrace_c.sh $1_old 1 && \
bash $R/profiles/scripts/ktrace_c.sh $1_new2 1 && \
VIHMC_LIB=$R/_var/$2 bash $R/profiles/scripts/ktrace_c.sh $1_old2 1
