# round 5: Gram form with the exact d ll / d b0 -- intermediates, the fit table with both dZb epilogue precisions,
# and the gradient-only class timing of the two epilogues
O=gpurun_out
for C in 1 16; do timeout -k 10 300 python -u profiles/scripts/diag/gram_parts_err.py 1e-2 $C || exit 1; done > $O/r05e_gram_parts.txt 2>&1
cat $O/r05e_gram_parts.txt
VIHMC_PARITY_CALIBRATE=1 VIHMC_PARITY_LOG=$O/r05e_parity.json timeout -k 10 600 python -u -m pytest tests/test_gpu_gram.py -m gpu -q -k "precision_vs_fit" --timeout 300 --timeout-method thread -p no:cacheprovider > $O/r05e_fit64.txt 2>&1
cp $O/gram_fit_table.json $O/r05e_fit_table_dzb64.json; rm -f $O/gram_fit_table.json
VIHMC_LIB=$PWD/_ab/dzb32.so VIHMC_PARITY_CALIBRATE=1 VIHMC_PARITY_LOG=$O/r05e_parity32.json timeout -k 10 600 python -u -m pytest tests/test_gpu_gram.py -m gpu -q -k "precision_vs_fit" --timeout 300 --timeout-method thread -p no:cacheprovider > $O/r05e_fit32.txt 2>&1
cp $O/gram_fit_table.json $O/r05e_fit_table_dzb32.json
for rep in 1 2; do for L in main dzb32; do
  echo "== $L rep $rep"
  VIHMC_LIB=$PWD/_ab/$L.so timeout -k 10 100 python -u profiles/scripts/probes/probe_classes.py --chains 16 --iters 30 --grad || exit 1
done; done > $O/r05e_dzb_ab.txt 2>&1
grep -v amdgpu.ids $O/r05e_dzb_ab.txt
