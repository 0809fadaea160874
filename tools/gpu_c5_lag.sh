#!/bin/bash
# Kind-22 wavefront lag at config 5's rank shape (n=4096, T_local=32, r=32) and
# at T_local=8: the stamped diagnostic build (tools/sweep_stamps.py --build
# --r=32 --tag=c5lag) records s_memrealtime at two step starts on every slice.
#   bash tools/gpu_c5_lag.sh TAG
set -o pipefail
TAG=${1:-c5lag}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export PYTHONUNBUFFERED=1
( while sleep 50; do date > $OUT/heartbeat; done ) &
HB=$!
timeout -k 10 300 python -u tools/sweep_stamps.py --tag=c5lag --n=4096 --T=32 --r=32 --kind=22 > $OUT/stamps_T32.txt 2>&1 &&
timeout -k 10 300 python -u tools/sweep_stamps.py --tag=c5lag --n=4096 --T=8 --r=32 --kind=22 > $OUT/stamps_T8.txt 2>&1
rc=$?
kill $HB
grep -h "wavefront\|mean step" $OUT/stamps_T32.txt $OUT/stamps_T8.txt
exit $rc
