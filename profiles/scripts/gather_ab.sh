#!/bin/bash
# Config 4's gradient gather at one chain: 169 full slices (1,020 parameters each, every thread busy) instead of 256
# slices of 673: the split / scale GPU tests with the variant, then the legs alternating _ab/base.so / _ab/g169.so.
TAG=${TAG:-r05g169}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
O=gpurun_out/${TAG}_ab.txt
mkdir -p gpurun_out
VIHMC_LIB=$ROOT/_ab/g169.so timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread -p no:cacheprovider \
    tests/test_gpu_scale_parity.py tests/test_gpu_split_fused.py > gpurun_out/${TAG}_tests.txt 2>&1
rc=$?; tail -3 gpurun_out/${TAG}_tests.txt; [ $rc -eq 0 ] || exit $rc
: > $O
for rep in 1 2 3; do
  for L in base g169; do
    echo "== $L rep $rep" >> $O
    VIHMC_LIB=$ROOT/_ab/$L.so timeout -k 10 150 python -u profiles/scripts/probes/probe_c4.py >> $O 2>/dev/null || exit 1
  done
done
python3 - $O <<'PY'
import json, sys
for line in open(sys.argv[1]):
    if line.startswith("=="): print(line.strip()); continue
    d = json.loads(line); print("  c4", round(d["leapfrog_steps_per_s"], 1), "half_eval_ms", round(d["ms_per_half_shard_eval"], 4))
PY
