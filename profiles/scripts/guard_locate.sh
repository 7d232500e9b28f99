# Out-of-bounds read locator (guard_poison.py), the normal GPU round (tests + bench), then the whole GPU suite under
# VIHMC_GUARD=1 (no -x: every test whose result depends on bytes behind a buffer). TAG names the outputs.
TAG=${TAG:-r04c}
timeout -k 10 300 python -u profiles/scripts/diag/guard_poison.py 80 > gpurun_out/${TAG}_poison.txt 2>&1 || exit $?
TAG=$TAG bash profiles/scripts/gpu_round.sh
VIHMC_GUARD=1 timeout -k 10 600 python -u -m pytest tests -m gpu -v --maxfail=25 --timeout 300 --timeout-method thread > gpurun_out/${TAG}_guard_tests.txt 2>&1
echo "guard tests rc=$?"; tail -3 gpurun_out/${TAG}_guard_tests.txt
