#!/bin/bash
# primitives + parity + bench + rocprof; stops at the first crash/hang
cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/${1:-v3b}; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 200 python -u -m pytest tests/test_gpu_primitives.py -x -v --timeout 120 --timeout-method thread > $OUT/prim.log 2>&1
rc=$?; echo "prim rc=$rc"; tail -3 $OUT/prim.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/gpu_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -15 $OUT/gpu_tests.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 300 python -u bench.py --no-cpu-baseline > $OUT/bench.json 2> $OUT/bench.err
rc=$?; echo "bench rc=$rc"; cat $OUT/bench.json; tail -5 $OUT/bench.err; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 -u bench.py --no-cpu-baseline --steps 5 --warmup 1 > $OUT/prof_bench.json 2> $OUT/prof.err
rc=$?; echo "prof rc=$rc"; head -8 $OUT/prof/run_kernel_stats.csv | cut -c1-150
