#!/bin/bash
# rocprofv3 kernel stats of a short bench run (timed region only) for each library named in LIBS (_ab/<name>.so;
# "main" = the in-tree build); prints the top kernels of each. Output: gpurun_out/${TAG}_<lib>_kstats.txt
TAG=${TAG:-r04kl}; LIBS=${LIBS:-main}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
O=$ROOT/gpurun_out
for L in $LIBS; do
  if [ "$L" = main ]; then LP=$ROOT/vi-hmc_amd/vihmc/libvihmc.so; else LP=$ROOT/_ab/$L.so; fi
  (cd /tmp && export TMPDIR=/tmp VIHMC_LIB=$LP VIHMC_ALLOW_DIAG=1 && timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv \
     -d $O/${TAG}_$L -o s -- python3 $ROOT/bench.py --steps 4 --warmup 1 --cpu-seconds 0 --no-side-legs --ess-steps 0 \
     > $O/${TAG}_$L.log 2>&1) || exit 1
  python3 $ROOT/profiles/kstats.py $(ls $O/${TAG}_$L/*kernel_stats.csv | head -1) 12 > $O/${TAG}_${L}_kstats.txt 2>&1
  echo "== $L"; cat $O/${TAG}_${L}_kstats.txt
done
