#!/bin/bash
# Rehearsal of the driver's torchrun bench on ONE GPU: 2 ranks (gloo; RCCL
# refuses two ranks per device), config 3 per-rank shape, per-rank timing and
# cross-rank wait accounting in the line.  Then N=1 with --force-dist (RCCL init).
set -o pipefail
TAG=${1:-r6tr}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/$TAG; mkdir -p $OUT
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
   --master-port 29533 bench.py --gpus 2 --steps 20 --warmup 3 --dist-backend gloo \
   > $OUT/bench_2rank_gloo.json 2> $OUT/bench_2rank_gloo.err || { echo "2-rank failed"; tail -30 $OUT/bench_2rank_gloo.err; exit 1; }
cat $OUT/bench_2rank_gloo.json | cut -c1-1500
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
   --master-port 29534 bench.py --gpus 1 --steps 20 --warmup 3 --force-dist \
   > $OUT/bench_1rank_nccl.json 2> $OUT/bench_1rank_nccl.err || { echo "1-rank nccl failed"; tail -30 $OUT/bench_1rank_nccl.err; exit 1; }
cat $OUT/bench_1rank_nccl.json | cut -c1-600
