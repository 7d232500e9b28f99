#!/bin/bash
# probe_classes alternating run-time settings, then one kernel trace per setting.
# Usage: bash profiles/scripts/ab_env_kt.sh <tag> "ENV=a" "ENV=b" ...
set -o pipefail
TAG=$1; shift
bash profiles/scripts/ab_env.sh $TAG "$@" || exit 1
i=0
for kv in "$@"; do
  bash profiles/scripts/ktrace.sh ${TAG}_$i $kv || exit 1
  i=$((i+1))
done
