mkdir -p gpurun_out
O=gpurun_out/r05ke_ab.txt
: > $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_sampler.py tests/test_gpu_split_fused.py tests/test_gpu_api.py tests/test_gpu_gram_traj.py tests/test_gpu_bench_path.py > gpurun_out/r05ke_tests.txt 2>&1 || exit 1
for rep in 1 2; do
  echo "== base rep $rep" >> $O
  SAMPLERS_FILE=$(pwd)/_ab/samplers_base.py timeout -k 10 200 python -u profiles/scripts/diag/legs_c1.py 1 >> $O 2>/dev/null || exit 1
  echo "== kinetic rep $rep" >> $O
  timeout -k 10 200 python -u profiles/scripts/diag/legs_c1.py 1 >> $O 2>/dev/null || exit 1
done
cat $O
