#!/bin/bash
# A chosen set of GPU tests in one process.  usage: tools/gpu_tests.sh TAG TIMEOUT_S TEST...
set -o pipefail
TAG=$1; TO=$2; shift 2
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/$TAG; mkdir -p $OUT
( while sleep 50; do date > $OUT/heartbeat; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
timeout -k 10 $TO python -u -m pytest -x -v --timeout 300 --timeout-method thread "$@" > $OUT/pytest.log 2>&1 \
  || { echo "pytest failed"; grep -E "FAILED|Error|error" $OUT/pytest.log | head -20; tail -40 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
