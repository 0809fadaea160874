#!/bin/bash
# quick loop: GPU parity (v3 path) + bench + stamps; stops at the first crash/hang
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/${1:-quick}; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/gpu_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -4 $OUT/gpu_tests.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 300 python -u bench.py --no-cpu-baseline > $OUT/bench.json 2> $OUT/bench.err
rc=$?; echo "bench rc=$rc"; python3 -c "import json;d=json.load(open('$OUT/bench.json'));print('ms/step',d['ms_per_step'],'kernels',d['kernels_ms'],'value %.3g'%d['value'])"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u tools/sweep3_stamps.py > $OUT/stamps.txt 2>&1; echo "stamps rc=$?"; cat $OUT/stamps.txt
