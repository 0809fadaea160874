#!/bin/bash
# Same-box A/B of two r=16 builds at config 3 for the three variants.  usage: TAG ROUNDS LIB_A LIB_B [LIB_C ...]
set -o pipefail
TAG=$1; ROUNDS=$2; shift 2
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/$TAG; mkdir -p $OUT
for V in good naive bad; do
  timeout -k 10 400 python -u tools/ab_v3.py "$@" --rounds $ROUNDS -- --steps 40 --warmup 5 --variant $V \
     > $OUT/ab_$V.txt 2>&1 || { echo "ab $V failed"; tail -30 $OUT/ab_$V.txt; exit 1; }
  echo "$V:"; grep median $OUT/ab_$V.txt
done
