#!/bin/bash
# Round-2 GPU pass: selected test files (or the whole -m gpu suite), then the bench line.
# usage: tools/gpu_r02.sh TAG "pytest-args" [bench]
set -o pipefail
TAG=${1:-r02}; TESTS=${2:-tests}; WHAT=${3:-bench}
OUT=gpurun_out/$TAG; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
if [[ $TESTS != none ]]; then
  timeout -k 10 900 python -u -m pytest $TESTS -m gpu -x -v --timeout 300 --timeout-method thread \
     > $OUT/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -40 $OUT/pytest_gpu.log; exit 1; }
  tail -3 $OUT/pytest_gpu.log
fi
if [[ $WHAT == bench ]]; then
  timeout -k 10 400 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed"; tail -30 $OUT/bench.err; exit 1; }
  cat $OUT/bench.json
fi
