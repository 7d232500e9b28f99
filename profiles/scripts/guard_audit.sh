# Bounds audit of reads: the GPU suites with every plan buffer ending at an unmapped guard granule (VIHMC_GUARD=1)
# and serialised kernel launches (the failing launch is the one reported). TAG names the outputs.
TAG=${TAG:-r04g}
export VIHMC_GUARD=1 AMD_SERIALIZE_KERNEL=3
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_gram.py tests/test_gpu_gram_traj.py tests/test_gpu_sampler.py -m gpu -v -x --timeout 300 --timeout-method thread > gpurun_out/${TAG}_guard_tests.txt 2>&1; rc=$?
echo "guard tests rc=$rc"; tail -5 gpurun_out/${TAG}_guard_tests.txt
exit $rc
