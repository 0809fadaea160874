#!/bin/bash
# Same-box A/B at config 3 plus a bit-equality check of the two builds' fit
# results (bench's elbo_last / mse_last, every variant).  usage: TAG ROUNDS LIB_A LIB_B
set -o pipefail
TAG=$1; ROUNDS=$2; A=$3; B=$4
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/$TAG; mkdir -p $OUT
for V in good naive bad; do
  for L in $A $B; do
    AME_LIB_PATH=$L timeout -k 10 200 python -u bench.py --no-cpu-baseline --steps 10 --warmup 2 --variant $V \
       > $OUT/eq_${V}_$(basename $L).json 2> $OUT/eq.err || { echo "bench $V $L failed"; tail -20 $OUT/eq.err; exit 1; }
  done
  python3 -c "
import json,sys
a=json.load(open('$OUT/eq_${V}_$(basename $A).json')); b=json.load(open('$OUT/eq_${V}_$(basename $B).json'))
print('$V', 'elbo', a['elbo_last'], b['elbo_last'], 'mse', a['mse_last'], b['mse_last'], 'EQUAL' if (a['elbo_last'],a['mse_last'])==(b['elbo_last'],b['mse_last']) else 'DIFFER')" || exit 1
done
bash tools/gpu_ab3v.sh $TAG $ROUNDS $A $B
