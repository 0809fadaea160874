#!/bin/bash
# Parity subset + rocprofv3 kernel statistics of the bench command.
# usage: tools/gpu_stats.sh TAG "pytest files"
set -o pipefail
TAG=${1:-stats}; TESTS=${2:-none}
OUT=gpurun_out/$TAG; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
if [[ $TESTS != none ]]; then
  timeout -k 10 600 python -u -m pytest $TESTS -m gpu -x -q --timeout 300 --timeout-method thread \
     > $OUT/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -40 $OUT/pytest_gpu.log; exit 1; }
  tail -2 $OUT/pytest_gpu.log
fi
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/stats -o run -- \
    python3 -u bench.py --no-cpu-baseline --steps 20 --warmup 5 > $OUT/stats_bench.json 2> $OUT/stats.err \
    || { echo "rocprof stats failed"; tail -20 $OUT/stats.err; exit 1; }
F=$(find $OUT/stats -name '*kernel_stats.csv' | head -1); cp $F $OUT/kernel_stats.csv
python3 -c "
import csv
for r in csv.DictReader(open('$OUT/kernel_stats.csv')):
    if 'ame_' in r['Name']: print(r['Name'][:60], r['Calls'], round(float(r['AverageNs'])/1e3,1), 'us')"
python3 -c "import json;d=json.load(open('$OUT/stats_bench.json'));print('ms/step',d['ms_per_step'])"
