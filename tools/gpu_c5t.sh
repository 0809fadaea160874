#!/bin/bash
# config-5 shape at T_local = 1, 8, 32 (v2 with GEMV workers): per node-step time, and stamps at T = 1
set -o pipefail
TAG=${1:-c5t}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/$TAG; mkdir -p $OUT; : > $OUT/c5t.jsonl
for T in 1 8 32; do
  timeout -k 10 300 python3 -u bench.py --no-cpu-baseline --steps 3 --warmup 1 --n 4096 --t-per-gpu $T --latent-dim 32 --variant good >> $OUT/c5t.jsonl 2> $OUT/err.log \
    || { echo "bench failed"; tail -20 $OUT/err.log; exit 1; }
  python3 -c "import json; z=[json.loads(l) for l in open('$OUT/c5t.jsonl')][-1]; print('T=$T', round(z['ms_per_step'],2), 'ms/iter', round(z['ms_per_step']*1000/4096,2), 'us/node-step')"
done
timeout -k 10 200 python -u tools/sweep_stamps.py --n=4096 --T=1 --r=32 2>&1 | grep -v amdgpu.ids > $OUT/stamps_T1.txt; cat $OUT/stamps_T1.txt
