#!/bin/bash
# (r05sp3: every job list, the one-chain legs too) k_reduce grid for the tiled dW jobs sized to their block need (16 chains: 11 x-blocks per job instead of 44, three
# quarters of them empty exits): GPU tests of the reduce paths, then the headline bench (no side legs) and the
# 16-chain gradient-only class timings alternating _ab/base.so / _ab/span.so.
TAG=${TAG:-r05sp3}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
O=gpurun_out/${TAG}_ab.txt
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -v --timeout 200 --timeout-method thread -p no:cacheprovider \
    tests/test_gpu_parity.py tests/test_gpu_bench_path.py tests/test_gpu_scale_parity.py \
    > gpurun_out/${TAG}_tests.txt 2>&1
rc=$?; tail -3 gpurun_out/${TAG}_tests.txt; [ $rc -eq 0 ] || exit $rc
: > $O
for rep in 1 2; do
  for L in base span; do
    echo "== $L rep $rep" >> $O
    VIHMC_LIB=$ROOT/_ab/$L.so timeout -k 10 200 python -u bench.py --cpu-seconds 0 --no-side-legs --ess-steps 0 >> $O 2>/dev/null || exit 1
    VIHMC_LIB=$ROOT/_ab/$L.so timeout -k 10 150 python -u profiles/scripts/probes/probe_legs.py --reps 1 >> $O 2>/dev/null || exit 1
  done
done
cd /tmp && export TMPDIR=/tmp
for L in base span; do
  VIHMC_LIB=$ROOT/_ab/$L.so timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $ROOT/gpurun_out/${TAG}_st_$L -o s -- \
      python3 $ROOT/bench.py --steps 40 --warmup 3 --cpu-seconds 0 --no-side-legs --ess-steps 0 > $ROOT/gpurun_out/${TAG}_st_$L.log 2>&1 || exit 1
  python3 $ROOT/profiles/kstats.py $(ls $ROOT/gpurun_out/${TAG}_st_$L/*kernel_stats.csv | head -1) 16 > $ROOT/gpurun_out/${TAG}_kstats_$L.txt 2>&1
  echo "== kstats $L"; grep -E "k_reduce|k_bwd_bf2|k_gather" $ROOT/gpurun_out/${TAG}_kstats_$L.txt
done
cd $ROOT
python3 - $O <<'PY'
import json, sys
for line in open(sys.argv[1]):
    if line.startswith("=="): print(line.strip()); continue
    try: d = json.loads(line)
    except Exception: continue
    if "metric" in d: print("  bench", round(d["value"], 1), "ms/step", round(d["ms_per_step"], 4), "sclk", round(d.get("sclk_mhz") or 0, 1))
    else: print("  legs", {k: round(v, 4) for k, v in d.items()})
PY
