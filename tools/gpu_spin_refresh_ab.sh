#!/bin/bash
# Kind 22 at config 5's rank shape: spin loops with (AME_SPIN_REFRESH=1) and
# without (=0) the periodic agent acquire.  Bit-equality of the two builds, the
# slice-start stamps with the refresh, then bench.py ms per iteration in
# alternating rounds (variant builds sr0 / sr1, r = 32).
#   bash tools/gpu_spin_refresh_ab.sh TAG
set -o pipefail
TAG=${1:-sr}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export PYTHONUNBUFFERED=1
( while sleep 50; do date > $OUT/heartbeat; done ) &
HB=$!
rc=0
for v in 0 1; do
    AME_LIB_PATH=tools/_lib/libame_amd_sr$v.so timeout -k 10 300 python -u tools/bitcmp.py save \
        $OUT/good$v.npz 600,8,32 good 3 22 >> $OUT/bitcmp.txt 2>&1 || { rc=1; break; }
done
[ $rc -eq 0 ] && { python tools/bitcmp.py cmp $OUT/good0.npz $OUT/good1.npz >> $OUT/bitcmp.txt 2>&1 || rc=1; }
if [ $rc -eq 0 ]; then
    timeout -k 10 300 python -u tools/sweep_stamps.py --tag=c5lagsr --n=4096 --T=32 --r=32 --kind=22 > $OUT/stamps1.txt 2>&1 &&
    timeout -k 10 300 python -u tools/sweep_stamps.py --tag=c5lagsr --n=4096 --T=32 --r=32 --kind=22 > $OUT/stamps2.txt 2>&1 &&
    timeout -k 10 900 python -u tools/ab_v3.py tools/_lib/libame_amd_sr0.so tools/_lib/libame_amd_sr1.so --rounds 4 -- \
        --n 4096 --t-per-gpu 32 --latent-dim 32 --steps 10 --warmup 2 --no-secondary > $OUT/ab.txt 2>&1
    rc=$?
fi
kill $HB
grep -h "EQUAL\|DIFF" $OUT/bitcmp.txt
grep -h "wavefront\|latest" $OUT/stamps*.txt
grep median $OUT/ab.txt
exit $rc
