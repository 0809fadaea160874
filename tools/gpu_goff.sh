#!/bin/bash
# v3 GEMV node->lane offset: parity, fit time per variant, stamp timelines.
set -o pipefail
OUT=gpurun_out/${1:-goff}; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_baseline_shapes.py -m gpu -x -q --timeout 300 --timeout-method thread \
   > $OUT/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
timeout -k 10 600 python -u tools/interference.py g0 g320 > $OUT/interference.txt 2>&1 || { echo "interference failed"; tail -20 $OUT/interference.txt; exit 1; }
cat $OUT/interference.txt
for T in "" g0; do
  timeout -k 10 120 python -u tools/sweep3_stamps.py --tag=$T > $OUT/stamps$T.txt 2>&1 || { echo "stamps failed"; tail -20 $OUT/stamps$T.txt; exit 1; }
  echo "== stamps $T"; head -40 $OUT/stamps$T.txt
done
