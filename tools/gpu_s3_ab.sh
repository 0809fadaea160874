#!/bin/bash
# v3 sweep: node i's old mean read at the step start (AME_S3_MOLD_EARLY) instead
# of in the publish; v3 parity with the product library, then same-box A/B at
# config 3 (variant builds s3m0 / s3m1, r = 16).
#   bash tools/gpu_s3_ab.sh TAG
set -o pipefail
TAG=${1:-s3}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export PYTHONUNBUFFERED=1
( while sleep 50; do date > $OUT/heartbeat; done ) &
HB=$!
timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread -p no:cacheprovider -m gpu \
    tests/test_gpu_parity.py tests/test_gpu_symmetry.py tests/test_gpu_stale_epoch.py > $OUT/pytest_v3.log 2>&1 &&
timeout -k 10 900 python -u tools/ab_v3.py ${S3_LIBS:-tools/_lib/libame_amd_s3m0.so tools/_lib/libame_amd_s3m1.so} \
    --rounds 5 -- --steps 30 --warmup 3 > $OUT/ab_c3.txt 2>&1
rc=$?
kill $HB
tail -2 $OUT/pytest_v3.log
grep median $OUT/ab_c3.txt
exit $rc
