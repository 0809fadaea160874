#!/bin/bash
# Same-box A/B at config 5's rank shape (r=32 variants).  usage: tools/gpu_ab5.sh TAG ROUNDS LIB...
set -o pipefail
TAG=$1; ROUNDS=$2; shift 2
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/$TAG; mkdir -p $OUT
timeout -k 10 900 python -u tools/ab_v3.py "$@" --rounds $ROUNDS -- --n 4096 --t-per-gpu 32 --latent-dim 32 \
   --steps 8 --warmup 2 > $OUT/ab_c5.txt 2>&1 || { echo "ab c5 failed"; tail -30 $OUT/ab_c5.txt; exit 1; }
grep median $OUT/ab_c5.txt
