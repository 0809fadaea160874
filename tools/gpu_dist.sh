#!/bin/bash
# Time-sharded ranks on one GPU (peer-buffer hand-off) + isolated ELBO kernels.
set -o pipefail
OUT=gpurun_out/${1:-dist}; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 700 python -u -m pytest tests/test_gpu_distributed.py tests/test_gpu_baseline_shapes.py -m gpu -x -v --timeout 300 --timeout-method thread \
   > $OUT/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -40 $OUT/pytest_gpu.log; exit 1; }
grep -E "PASSED|FAILED" $OUT/pytest_gpu.log | tail -12
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/stats -o run -- \
    python3 -u tools/elbo_iso.py > $OUT/iso.txt 2> $OUT/iso.err || { echo "iso failed"; tail -20 $OUT/iso.err; exit 1; }
F=$(find $OUT/stats -name '*kernel_stats.csv' | head -1); cp $F $OUT/kernel_stats.csv
python3 -c "
import csv
for r in csv.DictReader(open('$OUT/kernel_stats.csv')):
    if 'pairs' in r['Name'] or 'cov' in r['Name']: print(r['Name'][:40], r['Calls'], round(float(r['AverageNs'])/1e3,1), 'us')"
