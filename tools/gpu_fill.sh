#!/bin/bash
# Fill-bound regime on one GPU (short per-slice chain, many slices: the ratio of
# wavefront fill to chain that 8 time-sharded ranks have at config 3), depth 1/2/3
set -o pipefail
TAG=${1:-fill}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/$TAG; mkdir -p $OUT; : > $OUT/fill.txt
for N in 128 256; do for DP in 1 2 3; do
  AME_SPEC_DEPTH=$DP timeout -k 10 200 python3 -u bench.py --no-cpu-baseline --steps 40 --n $N --t-per-gpu 128 > $OUT/b.json 2> $OUT/err.log || { echo "bench failed"; tail -20 $OUT/err.log; exit 1; }
  python3 -c "import json; z=json.load(open('$OUT/b.json')); print('n=$N depth=$DP', round(z['ms_per_step'],3), '%.4g' % z['value'], {k: round(v,3) for k,v in z['kernels_ms'].items()})" | tee -a $OUT/fill.txt
done; done
