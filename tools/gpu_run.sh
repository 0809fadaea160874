#!/bin/bash
# Development pass on the GPU box: selected tests, then optional bench lines.
# usage: tools/gpu_run.sh TAG "pytest-args" ["bench args" ...]
#   each further argument is one bench.py invocation (its args), appended to bench.jsonl
set -o pipefail
TAG=${1:-run}; TESTS=${2:-}; shift 2
OUT=gpurun_out/$TAG; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
if [[ -n $TESTS ]]; then
  timeout -k 10 900 python -u -m pytest $TESTS -m gpu -x -v --timeout 200 --timeout-method thread \
     > $OUT/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -40 $OUT/pytest_gpu.log; exit 1; }
  tail -3 $OUT/pytest_gpu.log
fi
: > $OUT/bench.jsonl
for B in "$@"; do
  timeout -k 10 300 python3 -u bench.py $B >> $OUT/bench.jsonl 2> $OUT/bench.err \
    || { echo "bench $B failed"; tail -30 $OUT/bench.err; exit 1; }
  tail -1 $OUT/bench.jsonl | cut -c1-600
done
