# round 5: Gram form with fp64 Gt in the dZb epilogue and a four-plane -Gb: intermediates + gradient attribution, then
# the Gram GPU tests (calibration records) and the fit table
O=gpurun_out
for C in 1 16; do timeout -k 10 300 python -u profiles/scripts/diag/gram_parts_err.py 1e-2 $C || exit 1; done > $O/r05f_gram_parts.txt 2>&1
cat $O/r05f_gram_parts.txt | grep -v amdgpu.ids
rm -f $O/gram_fit_table.json
VIHMC_PARITY_CALIBRATE=1 VIHMC_PARITY_LOG=$O/r05f_parity.json timeout -k 10 900 python -u -m pytest tests/test_gpu_gram.py tests/test_gpu_gram_traj.py tests/test_gpu_bench_path.py -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider > $O/r05f_tests.txt 2>&1
tail -3 $O/r05f_tests.txt
cp $O/gram_fit_table.json $O/r05f_fit_table.json
for rep in 1 2; do
  timeout -k 10 100 python -u profiles/scripts/probes/probe_classes.py --chains 16 --iters 30 --grad || exit 1
done > $O/r05f_classes.txt 2>&1
grep -v amdgpu.ids $O/r05f_classes.txt
