#!/bin/bash
# Kind 22 (in-order GEMV workers) vs kind 23 (pipelined) at BASELINE config 5:
# per-rank shape (T = 32) and the full workload (T = 256), alternating runs.
set -o pipefail
TAG=${1:-pipeab}; ROUNDS=${2:-2}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/$TAG; mkdir -p $OUT
for r in $(seq $ROUNDS); do
  for K in 22 23; do
    timeout -k 10 200 python -u bench.py --n 4096 --t-per-gpu 32 --latent-dim 32 --no-cpu-baseline \
       --steps 10 --warmup 2 --sweep-kernel $K > $OUT/c5_k$K.r$r.json 2>> $OUT/err.log \
       || { echo "bench k$K failed"; tail $OUT/err.log; exit 1; }
    echo "rank shape kind $K round $r: $(grep -o '"ms_per_step": [0-9.]*' $OUT/c5_k$K.r$r.json)"
  done
done
for K in 22 23; do
  timeout -k 10 300 python -u bench.py --config5-full --sweep-kernel $K > $OUT/c5full_k$K.json 2>> $OUT/err.log \
     || { echo "config5-full k$K failed"; tail $OUT/err.log; exit 1; }
  echo "full kind $K: $(grep -o '"ms_per_iteration": [0-9.]*' $OUT/c5full_k$K.json | tr '\n' ' ')"
done
