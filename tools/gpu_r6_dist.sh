#!/bin/bash
# Multi-rank checks on one GPU: distributed / skew / slice-group tests, then the
# 2-rank gloo torchrun bench rehearsal.
set -o pipefail
TAG=${1:-r6d}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/$TAG; mkdir -p $OUT
timeout -k 10 700 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
   tests/test_gpu_distributed.py tests/test_gpu_skew.py \
   "tests/test_gpu_baseline_shapes.py::test_config4_full_T_one_gpu" \
   > $OUT/pytest.log 2>&1 || { echo "pytest failed"; tail -60 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
   --master-port 29533 bench.py --gpus 2 --steps 20 --warmup 3 --dist-backend gloo \
   > $OUT/bench_2rank_gloo.json 2> $OUT/bench_2rank_gloo.err || { echo "2-rank failed"; tail -30 $OUT/bench_2rank_gloo.err; exit 1; }
python3 -c "import json; z=json.loads(open('$OUT/bench_2rank_gloo.json').read().strip().splitlines()[-1]); print(z['ms_per_step'], z['per_rank_ms_per_step'], z['per_rank_cross_wait_ms_per_step'])"
