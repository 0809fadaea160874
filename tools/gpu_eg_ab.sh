#!/bin/bash
# Kind-22 partial gathers issued at the end of the previous step's phase 3
# (AME_EARLY_GATHER): v2 parity with the product library, then same-box A/B at
# config 5's rank shape (variant builds egoff / egon, r = 32).
#   bash tools/gpu_eg_ab.sh TAG
set -o pipefail
TAG=${1:-eg}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export PYTHONUNBUFFERED=1
( while sleep 50; do date > $OUT/heartbeat; done ) &
HB=$!
timeout -k 10 900 python -u -m pytest -x -v -s --timeout 900 --timeout-method thread -p no:cacheprovider -m gpu \
    tests/test_gpu_workers.py tests/test_gpu_large.py tests/test_gpu_w6_workers.py tests/test_gpu_config5_full.py \
    > $OUT/pytest_v2.log 2>&1 &&
timeout -k 10 600 python -u tools/ab_v3.py tools/_lib/libame_amd_egoff.so tools/_lib/libame_amd_egon.so \
    --rounds 3 -- --n 4096 --t-per-gpu 32 --latent-dim 32 --steps 10 --warmup 2 --no-secondary > $OUT/ab_c5.txt 2>&1
rc=$?
kill $HB
tail -3 $OUT/pytest_v2.log
grep median $OUT/ab_c5.txt
exit $rc
