#!/bin/bash
# v4 sweep bring-up: v4 parity tests, bench line, in-kernel stamp timeline.
# usage: tools/gpu_v4.sh TAG
set -o pipefail
TAG=${1:-v4}
OUT=gpurun_out/$TAG; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 600 python -u -m pytest tests/test_gpu_sweep4.py -m gpu -x -v --timeout 300 --timeout-method thread \
   > $OUT/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -2 $OUT/pytest_gpu.log
timeout -k 10 300 python -u bench.py --no-cpu-baseline > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed"; tail -30 $OUT/bench.err; exit 1; }
python -c "import json;d=json.load(open('$OUT/bench.json'));print('ms/step',d['ms_per_step'],'value',d['value'])"
timeout -k 10 300 python -u tools/sweep4_stamps.py > $OUT/stamps.txt 2>&1 || { echo "stamps failed"; tail -20 $OUT/stamps.txt; exit 1; }
cat $OUT/stamps.txt
