set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r02bq_gpu_tests.txt 2>&1 && \
bash profiles/scripts/ktrace_c.sh r02bq 1
