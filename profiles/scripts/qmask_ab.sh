#!/bin/bash
# Tiled dW slabs: only the quads that hold a sampled parameter stored / summed (ReduceJob::qmask). Tests with the
# in-tree library, then the headline bench (no side legs) and the one-chain legs alternating _ab/base.so / _ab/qm.so.
TAG=${TAG:-r05qm}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
O=gpurun_out/${TAG}_ab.txt
mkdir -p gpurun_out
export VIHMC_PARITY_LOG=$ROOT/gpurun_out/${TAG}_parity_errors.json
timeout -k 10 500 python -u -m pytest -x -v --timeout 200 --timeout-method thread -p no:cacheprovider \
    tests/test_gpu_parity.py tests/test_gpu_bench_path.py tests/test_gpu_scale_parity.py tests/test_gpu_gram.py \
    tests/test_gpu_sampler.py tests/test_gpu_gram_traj.py > gpurun_out/${TAG}_tests.txt 2>&1
rc=$?; tail -3 gpurun_out/${TAG}_tests.txt; [ $rc -eq 0 ] || exit $rc
: > $O
for rep in 1 2; do
  for L in base qm; do
    echo "== $L rep $rep" >> $O
    VIHMC_LIB=$ROOT/_ab/$L.so timeout -k 10 200 python -u bench.py --cpu-seconds 0 --no-side-legs --ess-steps 0 >> $O 2>/dev/null || exit 1
    VIHMC_LIB=$ROOT/_ab/$L.so timeout -k 10 150 python -u profiles/scripts/probes/probe_legs.py --reps 1 >> $O 2>/dev/null || exit 1
  done
done
python3 - $O <<'PY'
import json, sys
for line in open(sys.argv[1]):
    if line.startswith("=="): print(line.strip()); continue
    try: d = json.loads(line)
    except Exception: continue
    if "metric" in d: print("  bench", round(d["value"], 1), "ms/step", round(d["ms_per_step"], 4), "bwd_us", round(d["roofline"]["avg_launch_ms"] * 1e3, 2))
    else: print("  legs", {k: round(v, 4) for k, v in d.items()})
PY
