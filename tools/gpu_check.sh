#!/bin/bash
# One GPU-box pass: parity tests, bench (with CPU baseline), rocprof kernel stats.
# usage: tools/gpu_check.sh TAG [tests|bench|prof|all]
set -o pipefail
TAG=${1:-run}; WHAT=${2:-all}
OUT=gpurun_out/$TAG; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
if [[ $WHAT == all || $WHAT == tests ]]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
     > $OUT/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 $OUT/pytest_gpu.log; exit 1; }
  tail -3 $OUT/pytest_gpu.log
fi
if [[ $WHAT == all || $WHAT == bench ]]; then
  timeout -k 10 300 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed"; tail -30 $OUT/bench.err; exit 1; }
  cat $OUT/bench.json
fi
if [[ $WHAT == all || $WHAT == prof ]]; then
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- \
     python3 -u bench.py --no-cpu-baseline --steps 5 --warmup 1 > $OUT/prof_bench.json 2> $OUT/prof.err \
     || { echo "rocprof failed"; tail -30 $OUT/prof.err; exit 1; }
  find $OUT/prof -name '*kernel_stats.csv' | head -3
fi
