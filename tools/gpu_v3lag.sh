#!/bin/bash
# v3 with / without the forced slice lag: bench (v3 forced) + stamp timelines.
set -o pipefail
OUT=gpurun_out/${1:-v3lag}; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1

timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 20 --warmup 5 > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed"; tail -30 $OUT/bench.err; exit 1; }
python -c "import json;d=json.load(open('$OUT/bench.json'));print('v3+lag ms/step',d['ms_per_step'])"
for T in "" _nolag _lag3; do
  timeout -k 10 200 python -u tools/sweep3_stamps.py --tag=$T > $OUT/stamps$T.txt 2>&1 || { echo "stamps $T failed"; tail -20 $OUT/stamps$T.txt; exit 1; }
  echo "== $T"; grep "step period" $OUT/stamps$T.txt; grep -A3 "per-lane elapsed" $OUT/stamps$T.txt | tail -1
done
