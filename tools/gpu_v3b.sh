#!/bin/bash
# v3 solver-side v/yv (HF2 removed): parity tests, bench, stamp timeline.
set -o pipefail
OUT=gpurun_out/${1:-v3b}; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_baseline_shapes.py > $OUT/pytest.txt 2>&1 || { echo "pytest failed"; tail -30 $OUT/pytest.txt; exit 1; }
tail -2 $OUT/pytest.txt
timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 20 --warmup 5 > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed"; tail -30 $OUT/bench.err; exit 1; }
python -c "import json;d=json.load(open('$OUT/bench.json'));print('ms/step',d['ms_per_step'], d['kernels'])"
timeout -k 10 200 python -u tools/sweep3_stamps.py > $OUT/stamps.txt 2>&1 || { echo "stamps failed"; tail -20 $OUT/stamps.txt; exit 1; }
cat $OUT/stamps.txt
