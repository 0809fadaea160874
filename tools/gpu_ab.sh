#!/bin/bash
# Same-box A/B of variant libraries (tools/ab_v3.py) on the config-3 bench.
# usage: tools/gpu_ab.sh TAG ROUNDS LIB...
set -o pipefail
TAG=$1; ROUNDS=$2; shift 2
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/$TAG; mkdir -p $OUT
timeout -k 10 900 python -u tools/ab_v3.py "$@" --rounds $ROUNDS -- --steps 40 --warmup 5 > $OUT/ab.txt 2>&1 \
   || { echo "ab failed"; tail -30 $OUT/ab.txt; exit 1; }
tail -n $(( $# )) $OUT/ab.txt
