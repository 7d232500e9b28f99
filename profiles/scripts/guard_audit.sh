# Bounds audit of reads: the whole GPU suite with every plan buffer ending at an unmapped guard granule (VIHMC_GUARD=1),
# then the normal GPU round (tests + bench) when it is green. TAG names the outputs.
TAG=${TAG:-r04g}
VIHMC_GUARD=1 timeout -k 10 600 python -u -m pytest tests -m gpu -v -x --timeout 300 --timeout-method thread > gpurun_out/${TAG}_guard_tests.txt 2>&1; rc=$?
echo "guard tests rc=$rc"; tail -3 gpurun_out/${TAG}_guard_tests.txt
[ $rc -ne 0 ] && exit $rc
TAG=$TAG bash profiles/scripts/gpu_round.sh
rc=$?
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u profiles/scripts/probes/probe_groups.py --groups 1 2 4 --steps 20 --reps 2 > gpurun_out/${TAG}_groups.txt 2>&1
