#!/bin/bash
# Kind-22 wavefront fill: config 5's per-rank shape at T_local = 1, 8, 32
# (per-iteration time vs T_local; the slope over slices / the node step = F).
set -o pipefail
TAG=${1:-c5fill}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/$TAG; mkdir -p $OUT
for TLOC in 1 8 32; do
  timeout -k 10 200 python -u bench.py --n 4096 --t-per-gpu $TLOC --latent-dim 32 --no-cpu-baseline \
     --steps 8 --warmup 2 >> $OUT/c5_fill.jsonl 2>> $OUT/c5_fill.err || { echo "bench T=$TLOC failed"; tail $OUT/c5_fill.err; exit 1; }
done
grep -o '"ms_per_step": [0-9.]*' $OUT/c5_fill.jsonl
