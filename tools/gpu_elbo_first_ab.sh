#!/bin/bash
# Config 5's rank shape (kind 22): this iteration's ELBO queued before the
# speculative next sweep (elbo_first, on) or after it (off).  Parity of the two
# orders, the per-slice start stamps with the new order, then bench.py ms per
# iteration in alternating rounds.
#   bash tools/gpu_elbo_first_ab.sh TAG
set -o pipefail
TAG=${1:-ef}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export PYTHONUNBUFFERED=1
( while sleep 50; do date > $OUT/heartbeat; done ) &
HB=$!
timeout -k 10 600 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread -p no:cacheprovider \
    -m gpu tests/test_gpu_w6_workers.py -k "elbo_first or small_bit_equal" > $OUT/pytest_ef.log 2>&1 &&
timeout -k 10 300 python -u tools/sweep_stamps.py --tag=c5lag --n=4096 --T=32 --r=32 --kind=22 > $OUT/stamps_on.txt 2>&1
rc=$?
if [ $rc -eq 0 ]; then
  ARGS="--n 4096 --t-per-gpu 32 --latent-dim 32 --steps 10 --warmup 2 --no-cpu-baseline --no-secondary"
  for rnd in 1 2 3 4; do
    for cfg in off on; do
      timeout -k 10 300 python -u bench.py $ARGS --elbo-first $cfg > $OUT/b_${cfg}_$rnd.json 2> $OUT/b_${cfg}_$rnd.err || { rc=1; break 2; }
      python3 -c "import json,sys; b=json.loads(open('$OUT/b_${cfg}_$rnd.json').read().strip().splitlines()[-1]); print('$cfg round $rnd', round(b['ms_per_step'],3), b['config'].get('sweep_kind'), b['schedule'])" | tee -a $OUT/ab.txt
    done
  done
fi
kill $HB
tail -3 $OUT/pytest_ef.log
grep -h wavefront $OUT/stamps_on.txt
exit $rc
