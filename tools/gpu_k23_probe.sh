#!/bin/bash
# Kind 22 vs kind 23 per-iteration time at smaller n (variant r=32 libraries)
set -o pipefail
TAG=${1:-k23probe}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/$TAG; mkdir -p $OUT
run() {  # lib kind n T
  AME_LIB_PATH=$PWD/tools/_lib/libame_amd_$1.so timeout -k 10 120 python -u bench.py --n $3 --t-per-gpu $4 \
    --latent-dim 32 --no-cpu-baseline --steps 6 --warmup 2 --sweep-kernel $2 > $OUT/$1_k$2_n$3_T$4.json 2>> $OUT/err.log \
    || { echo "failed $1 $2 $3 $4"; tail -5 $OUT/err.log; exit 1; }
  echo "$1 kind $2 n=$3 T=$4: $(grep -o '"ms_per_step": [0-9.]*' $OUT/$1_k$2_n$3_T$4.json)"
}
for r in 1 2; do
  run base32 22 4096 32; run b152 22 4096 32; run b152 23 4096 32; run b224 23 4096 32
  run b152 23 4096 16; run b224 23 4096 16
done
