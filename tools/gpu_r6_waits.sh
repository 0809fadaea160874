#!/bin/bash
# Round 6: the wait rules (status block, no-progress budget, co-residency per
# shared GPU) on the GPU, then a same-box A/B of the r=16 v3 build against HEAD.
# usage: tools/gpu_r6_waits.sh TAG
set -o pipefail
TAG=${1:-r6w}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/$TAG; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
   tests/test_gpu_skew.py tests/test_gpu_stale_epoch.py \
   "tests/test_gpu_baseline_shapes.py::test_config4_full_T_one_gpu" \
   "tests/test_gpu_baseline_shapes.py::test_config4_rank_shape_two_ranks" \
   > $OUT/pytest_waits.log 2>&1 || { echo "pytest failed"; tail -60 $OUT/pytest_waits.log; exit 1; }
tail -3 $OUT/pytest_waits.log
timeout -k 10 400 python -u tools/ab_v3.py tools/_lib/libame_amd_r5head.so tools/_lib/libame_amd_r6new.so \
   --rounds 5 -- --steps 40 --warmup 5 > $OUT/ab.txt 2>&1 || { echo "ab failed"; tail -30 $OUT/ab.txt; exit 1; }
tail -3 $OUT/ab.txt
