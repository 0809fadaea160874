#!/bin/bash
# Per-iteration time vs iterations per fit() call (fill / per-call overhead).
set -o pipefail
TAG=${1:-steps}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/$TAG; mkdir -p $OUT; : > $OUT/s.txt
for T in 128 64; do for K in 5 10 20 40; do
  timeout -k 10 200 python3 -u bench.py --no-cpu-baseline --steps $K --warmup 2 --t-per-gpu $T > $OUT/one.json 2> $OUT/err.log \
    || { echo "bench failed"; tail -20 $OUT/err.log; exit 1; }
  python3 -c "import json,sys; z=json.load(open('$OUT/one.json')); print('T=$T K=$K', round(z['ms_per_step'],3), {k: round(v,3) for k,v in z['kernels_ms'].items()})" | tee -a $OUT/s.txt
done; done
