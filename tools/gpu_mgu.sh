#!/bin/bash
# config 5 per rank (n=4096, T=32, r=32, good): GEMV rows in flight per thread (AME_MG_UNROLL 8/16/32)
set -o pipefail
TAG=${1:-mgu}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/$TAG; mkdir -p $OUT; : > $OUT/mgu.txt
B=python-temporal-ame-svi_amd/ame_amd
for L in libame_amd.so _build/libame_amd_u16.so _build/libame_amd_u32.so; do
  AME_LIB_PATH=$GRAFT_REPO_ROOT/$B/$L timeout -k 10 300 python3 -u bench.py --no-cpu-baseline --steps 3 --warmup 1 --n 4096 --t-per-gpu 32 --latent-dim 32 > $OUT/b.json 2> $OUT/err.log || { echo "bench failed"; tail -20 $OUT/err.log; exit 1; }
  python3 -c "import json; z=json.load(open('$OUT/b.json')); print('$L', round(z['ms_per_step'],2), {k: round(v,2) for k,v in z['kernels_ms'].items()})" | tee -a $OUT/mgu.txt
done
