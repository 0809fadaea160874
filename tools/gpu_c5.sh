#!/bin/bash
# v2 wide / HBM-slice / GEMV-worker parity, then config 5 per-rank timing
# (naive/good/bad with workers; good without).
set -o pipefail
TAG=${1:-c5}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/$TAG; mkdir -p $OUT; : > $OUT/c5.jsonl
timeout -k 10 600 python -u -m pytest tests/test_gpu_workers.py tests/test_gpu_large.py -x -v --timeout 300 --timeout-method thread > $OUT/large.log 2>&1 \
  || { echo "tests failed"; tail -30 $OUT/large.log; exit 1; }
tail -2 $OUT/large.log
run() {  # variant, extra env
  env $2 timeout -k 10 300 python3 -u bench.py --no-cpu-baseline --steps 3 --warmup 1 --n 4096 --t-per-gpu 32 --latent-dim 32 --variant $1 >> $OUT/c5.jsonl 2> $OUT/err.log \
    || { echo "bench failed"; tail -20 $OUT/err.log; exit 1; }
  python3 -c "import json; z=[json.loads(l) for l in open('$OUT/c5.jsonl')][-1]; print('$1 $2', round(z['ms_per_step'],2), 'ms/iter', round(z['ms_per_step']*1000/4096,2), 'us/node-step', z['config'].get('sweep_kind'))"
}
for V in naive good bad; do run $V "X=1" || exit 1; done
# (single-workgroup v2 for comparison: run good "AME_SWEEP_NOWORKERS=1")
