#!/bin/bash
# side-A stamps: full kernel, no D MFMAs (CB_ABL=2), no S MFMAs (CB_ABL=3). Usage: stamps_a_abl.sh <tag>
TAG=$1
mkdir -p gpurun_out
for v in cbstamp cbst_nod cbst_nos; do
  VIHMC_ALLOW_DIAG=1 VIHMC_LIB=$PWD/_var/$v.so timeout -k 10 120 python profiles/scripts/diag/stamps_side_a.py \
      > gpurun_out/${TAG}_$v.log 2>&1 || exit 1
done
