#!/bin/bash
# primitives self-test, then parity (only if the first step did not crash/hang)
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/${1:-v3a}; mkdir -p $OUT
timeout -k 10 200 python -u -m pytest tests/test_gpu_primitives.py -x -v --timeout 120 --timeout-method thread > $OUT/prim.log 2>&1
rc=$?; echo "prim rc=$rc"; tail -5 $OUT/prim.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 120 --timeout-method thread > $OUT/parity.log 2>&1
rc=$?; echo "parity rc=$rc"; tail -40 $OUT/parity.log; exit $rc
