#!/bin/bash
# Same-box A/B: config 3 (r=16 variants) and config 5's rank shape (r=32 variants).
# usage: tools/gpu_ab2.sh TAG "LIBS16" "LIBS32"
set -o pipefail
TAG=$1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/$TAG; mkdir -p $OUT
timeout -k 10 500 python -u tools/ab_v3.py $2 --rounds 5 -- --steps 40 --warmup 5 > $OUT/ab_c3.txt 2>&1 \
   || { echo "ab c3 failed"; tail -30 $OUT/ab_c3.txt; exit 1; }
grep median $OUT/ab_c3.txt
timeout -k 10 500 python -u tools/ab_v3.py $3 --rounds 3 -- --n 4096 --t-per-gpu 32 --latent-dim 32 --steps 8 --warmup 2 \
   > $OUT/ab_c5.txt 2>&1 || { echo "ab c5 failed"; tail -30 $OUT/ab_c5.txt; exit 1; }
grep median $OUT/ab_c5.txt
