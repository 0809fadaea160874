#!/bin/bash
# Kind-22 phase 3 in blocks (AME_PH3_BLOCK): parity of the v2 kernels with the
# product library, then same-box A/B at config 5's rank shape (variant builds
# ph3old / ph3new, r = 32) through bench.py.
#   bash tools/gpu_ph3_ab.sh TAG
set -o pipefail
TAG=${1:-ph3}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export PYTHONUNBUFFERED=1
# heartbeat: long CPU-side oracle replays print nothing for minutes
( while sleep 50; do date > $OUT/heartbeat; done ) &
HB=$!
PT="python -u -m pytest -x -v --timeout 900 --timeout-method thread -p no:cacheprovider"
timeout -k 10 900 $PT -s -m gpu tests/test_gpu_workers.py tests/test_gpu_large.py \
    tests/test_gpu_pipe_workers.py tests/test_gpu_config5_full.py > $OUT/pytest_v2.log 2>&1 &&
timeout -k 10 600 python -u tools/ab_v3.py tools/_lib/libame_amd_ph3old.so tools/_lib/libame_amd_ph3new.so \
    --rounds 3 -- --n 4096 --t-per-gpu 32 --latent-dim 32 --steps 8 --warmup 2 --no-secondary > $OUT/ab_c5.txt 2>&1
rc=$?
kill $HB
tail -3 $OUT/pytest_v2.log
grep median $OUT/ab_c5.txt
exit $rc
