#!/bin/bash
# Round 6: MFMA P_0 sums in the sweep prologues -- parity tests on the product
# build, then same-box A/Bs (config 3 r=16 variants, config 5 rank shape r=32).
set -o pipefail
TAG=${1:-r6p}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/$TAG; mkdir -p $OUT
timeout -k 10 700 python -u -m pytest -x -v --timeout 400 --timeout-method thread \
   tests/test_gpu_parity.py tests/test_gpu_workers.py \
   "tests/test_gpu_baseline_shapes.py::test_config3_schedule_prefix_and_elbo" \
   "tests/test_gpu_baseline_shapes.py::test_config5_rank_shape" \
   > $OUT/pytest.log 2>&1 || { echo "pytest failed"; tail -60 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
L=tools/_lib
timeout -k 10 500 python -u tools/ab_v3.py $L/libame_amd_r5head.so $L/libame_amd_r6new.so $L/libame_amd_v2simple.so \
   $L/libame_amd_v3notag.so $L/libame_amd_v4both.so $L/libame_amd_r6mfma.so --rounds 4 -- --steps 40 --warmup 5 \
   > $OUT/ab_c3.txt 2>&1 || { echo "ab c3 failed"; tail -30 $OUT/ab_c3.txt; exit 1; }
tail -6 $OUT/ab_c3.txt
timeout -k 10 400 python -u tools/ab_v3.py $L/libame_amd_r5head32.so $L/libame_amd_r6mfma32.so --rounds 3 -- \
   --n 4096 --t-per-gpu 32 --latent-dim 32 --steps 8 --warmup 2 > $OUT/ab_c5.txt 2>&1 \
   || { echo "ab c5 failed"; tail -30 $OUT/ab_c5.txt; exit 1; }
tail -2 $OUT/ab_c5.txt
