#!/bin/bash
# Forward W-fragment prefetch A/B (round 4): bitwise dumps of the product build vs FWD_PIPE=0 (_ab/base.so)
# and the 8-wave variant (_ab/fw8.so), forward stamps at one chain, gradient-only class timings at 16 chains,
# and the one-chain crossover. Output: gpurun_out/${TAG}.txt
TAG=${TAG:-r04zf}
O=gpurun_out/${TAG}.txt
D=${GRAFT_REPO_ROOT:-$(pwd)}/_ab
VIHMC_LIB=$D/base.so timeout -k 10 100 python -u profiles/scripts/diag/dump_eval.py gpurun_out/dump_base.npz > $O 2>&1 || exit 1
timeout -k 10 100 python -u profiles/scripts/diag/dump_eval.py gpurun_out/dump_new.npz >> $O 2>&1 || exit 1
python profiles/scripts/diag/dump_eval.py --compare gpurun_out/dump_base.npz gpurun_out/dump_new.npz >> $O 2>&1
if [ -f $D/fw8.so ]; then
  VIHMC_LIB=$D/fw8.so timeout -k 10 100 python -u profiles/scripts/diag/dump_eval.py gpurun_out/dump_fw8.npz >> $O 2>&1 || exit 1
  python profiles/scripts/diag/dump_eval.py --compare gpurun_out/dump_base.npz gpurun_out/dump_fw8.npz >> $O 2>&1
fi
VIHMC_ALLOW_DIAG=1 VIHMC_LIB=$D/fwstamp.so timeout -k 10 120 python -u profiles/scripts/diag/stamps_fwd.py --chains 1 >> $O 2>&1 || exit 1
for L in base fw8; do
  [ -f $D/$L.so ] || continue
  echo "== $L" >> $O
  VIHMC_LIB=$D/$L.so timeout -k 10 100 python -u profiles/scripts/probes/probe_classes.py --chains 16 --iters 30 --grad >> $O 2>&1 || exit 1
done
echo "== product" >> $O
timeout -k 10 100 python -u profiles/scripts/probes/probe_classes.py --chains 16 --iters 30 --grad >> $O 2>&1 || exit 1
timeout -k 10 200 python -u profiles/scripts/probes/probe_crossover.py --chains 1 --rows 1000 500 >> $O 2>&1 || exit 1
grep -v amdgpu.ids $O
