#!/bin/bash
# One GPU call: GPU parity tests of the in-tree build and of each A/B variant (a test FAILURE is reported and
# the call goes on; a timeout / abort / fault ends it), then per-kernel stats of base + variants
# (profiles/ab_kstats.sh). Usage: bash profiles/ab_parity_then_stats.sh <tag> <variant.so> ...
TAG=$1; shift
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
O=$ROOT/gpurun_out/$TAG
mkdir -p $O
step() {   # step <log> <cmd...>: rc 0/1 (pass / test failure) continue, anything else stops the call
    local log=$1; shift
    timeout -k 10 300 "$@" > $log 2>&1
    local rc=$?
    echo "rc=$rc $log" >> $O/steps.txt
    [ $rc -le 1 ] || exit $rc
}
T="python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_api.py tests/test_gpu_sampler.py -x -q --timeout 120 --timeout-method thread"
step $O/par_base.log $T
for v in "$@"; do
    VIHMC_LIB=$ROOT/_var/$v step $O/par_$v.log $T
done
args=(base)
for v in "$@"; do args+=($v); done
bash $ROOT/profiles/ab_kstats.sh $TAG "${args[@]}" "${args[@]}"
