#!/bin/bash
# ab_side_a.sh plus side-A stamps of _var/cbstamp.so. Usage: ab_side_a_st.sh <tag> <variant> ...
set -o pipefail
TAG=$1
bash profiles/scripts/ab_side_a.sh "$@" && \
VIHMC_ALLOW_DIAG=1 VIHMC_LIB=$PWD/_var/cbstamp.so timeout -k 10 120 python profiles/scripts/diag/stamps_side_a.py \
    > gpurun_out/${TAG}_stamps_a.log 2>&1
