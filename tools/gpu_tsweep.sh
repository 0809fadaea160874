#!/bin/bash
# Per-iteration time vs slices per GPU at n=1024, r=16 (pipelined and in-order).
set -o pipefail
TAG=${1:-tsweep}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/$TAG; mkdir -p $OUT; : > $OUT/t.jsonl
for P in 1 0; do for T in 32 64 96 128; do
  AME_PIPELINE=$P timeout -k 10 200 python3 -u bench.py --no-cpu-baseline --steps 10 --warmup 2 --t-per-gpu $T > $OUT/one.json 2> $OUT/err.log \
    || { echo "bench T=$T failed"; tail -20 $OUT/err.log; exit 1; }
  python3 -c "import json,sys; z=json.load(open('$OUT/one.json')); print('P=$P T=$T', round(z['ms_per_step'],3), {k: round(v,3) for k,v in z['kernels_ms'].items()})" | tee -a $OUT/t.jsonl
done; done
