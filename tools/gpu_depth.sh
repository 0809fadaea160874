#!/bin/bash
# speculation depth: parity/exactness tests, then N=1 bench at depth 1 / 2 / 3
set -o pipefail
TAG=${1:-depth}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/$TAG; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/t.log 2>&1 \
  || { echo "tests failed"; tail -30 $OUT/t.log; exit 1; }
tail -1 $OUT/t.log
for DP in 1 2 3; do for K in 10 40; do
  AME_SPEC_DEPTH=$DP timeout -k 10 200 python3 -u bench.py --no-cpu-baseline --steps $K > $OUT/b.json 2> $OUT/err.log || { echo "bench failed"; tail -20 $OUT/err.log; exit 1; }
  python3 -c "import json; z=json.load(open('$OUT/b.json')); print('depth=$DP K=$K', round(z['ms_per_step'],3), '%.4g' % z['value'], {k: round(v,3) for k,v in z['kernels_ms'].items()})"
done; done
