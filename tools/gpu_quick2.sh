#!/bin/bash
# parity + bench (10 and 40 iterations) + stamp timeline
set -o pipefail
TAG=${1:-q2}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/$TAG; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_distributed.py -x -q --timeout 300 --timeout-method thread > $OUT/t.log 2>&1 \
  || { echo "tests failed"; tail -30 $OUT/t.log; exit 1; }
tail -1 $OUT/t.log
for K in 10 40; do
  timeout -k 10 200 python3 -u bench.py --no-cpu-baseline --steps $K > $OUT/b$K.json 2> $OUT/err.log || { echo "bench failed"; tail -20 $OUT/err.log; exit 1; }
  python3 -c "import json; z=json.load(open('$OUT/b$K.json')); print('K=$K', round(z['ms_per_step'],3), '%.4g' % z['value'], {k: round(v,3) for k,v in z['kernels_ms'].items()})"
done
timeout -k 10 200 python3 -u tools/sweep3_stamps.py > $OUT/stamps.txt 2>&1 || { echo "stamps failed"; tail $OUT/stamps.txt; exit 1; }
grep -v amdgpu.ids $OUT/stamps.txt | head -34
