#!/bin/bash
# BASELINE configs other than the headline one, one GPU's share each:
# config 2 (n=256, T=64, r=8), config 4 per rank (n=1024, T=64, r=16),
# config 3's shape with the naive and bad variants, config 5 per rank
# (n=4096, T=32, r=32; naive / good / bad).
# usage: tools/gpu_configs.sh TAG
set -o pipefail
TAG=${1:-configs}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/$TAG; mkdir -p $OUT; : > $OUT/configs.jsonl
run() {
  timeout -k 10 300 python3 -u bench.py --no-cpu-baseline "$@" >> $OUT/configs.jsonl 2> $OUT/err.log \
    || { echo "bench $* failed"; tail -20 $OUT/err.log; exit 1; }
  tail -1 $OUT/configs.jsonl | cut -c1-400
}
run --steps 30 --warmup 3 --n 256 --t-per-gpu 64 --latent-dim 8
run --steps 30 --warmup 3 --n 1024 --t-per-gpu 64 --latent-dim 16
for V in naive bad; do run --steps 30 --warmup 3 --variant $V; done
for V in naive good bad; do run --steps 10 --warmup 2 --n 4096 --t-per-gpu 32 --latent-dim 32 --variant $V; done
