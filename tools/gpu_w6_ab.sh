#!/bin/bash
# Six-worker sweep (kind 24) and the ELBO beside the sweep (elbo_cus): parity,
# then config 5's rank shape, rounds alternating kind 22 / kind 24 / kind 24 +
# ELBO on 32 CUs (bench.py ms per iteration).
#   bash tools/gpu_w6_ab.sh TAG
set -o pipefail
TAG=${1:-w6}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export PYTHONUNBUFFERED=1
( while sleep 50; do date > $OUT/heartbeat; done ) &
HB=$!
timeout -k 10 900 python -u -m pytest -x -v -s --timeout 600 --timeout-method thread -p no:cacheprovider \
    -m gpu tests/test_gpu_w6_workers.py ${W6_TESTS:+-k "$W6_TESTS"} > $OUT/pytest_w6.log 2>&1
rc=$?
if [ $rc -eq 0 ]; then
  ARGS="--n 4096 --t-per-gpu 32 --latent-dim 32 --steps 10 --warmup 2 --no-cpu-baseline --no-secondary"
  for rnd in 1 2 3; do
    for cfg in "k22:" "k24:--sweep-kernel 24" "k24cu:--sweep-kernel 24 --elbo-cus 32"; do
      name=${cfg%%:*}; extra=${cfg#*:}
      timeout -k 10 300 python -u bench.py $ARGS $extra > $OUT/b_${name}_$rnd.json 2> $OUT/b_${name}_$rnd.err || { rc=1; break 2; }
      python3 -c "import json,sys; b=json.loads(open('$OUT/b_${name}_$rnd.json').read().strip().splitlines()[-1]); print('$name round $rnd', round(b['ms_per_step'],3), b['config'].get('sweep_kind'), b['config'].get('elbo_cus'))" | tee -a $OUT/ab.txt
    done
  done
fi
kill $HB
tail -3 $OUT/pytest_w6.log
exit $rc
