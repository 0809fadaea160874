#!/bin/bash
# Round-end check: full GPU suite, smoke(), then the profile script.
set -o pipefail
TAG=${1:-final}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/$TAG; mkdir -p $OUT
# heartbeat: single tests (config 5's full workload) run longer than gpurun's 180 s silence limit
( while sleep 50; do date > $OUT/heartbeat; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 \
  || { echo "pytest failed"; tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo "smoke failed"; tail $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
bash tools/gpu_profile.sh $TAG
