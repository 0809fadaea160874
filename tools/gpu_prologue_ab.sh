#!/bin/bash
# v2 sweep prologue: P_0's node sums staged through LDS (HEAD) vs the direct
# per-entry HBM walk (tools/_lib/libame_amd_before.so).  Bit-equality of the
# two builds (kinds 21, 22), the slice-start stamps, the kind-22 GPU tests, and
# bench.py ms per iteration at config 5's rank shape in alternating rounds.
#   bash tools/gpu_prologue_ab.sh TAG
set -o pipefail
TAG=${1:-p0}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export PYTHONUNBUFFERED=1
( while sleep 50; do date > $OUT/heartbeat; done ) &
HB=$!
NEW=python-temporal-ame-svi_amd/ame_amd/libame_amd.so
OLD=tools/_lib/libame_amd_before.so
rc=0
for cfg in "600,8,32 good 3 22" "600,8,32 naive 3 22" "600,8,32 bad 3 22" "1024,4,16 good 3 21"; do
    name=$(echo $cfg | tr ' ,' '__')
    AME_LIB_PATH=$OLD timeout -k 10 300 python -u tools/bitcmp.py save $OUT/o_$name.npz $cfg >> $OUT/bitcmp.txt 2>&1 &&
    AME_LIB_PATH=$NEW timeout -k 10 300 python -u tools/bitcmp.py save $OUT/n_$name.npz $cfg >> $OUT/bitcmp.txt 2>&1 &&
    python tools/bitcmp.py cmp $OUT/o_$name.npz $OUT/n_$name.npz >> $OUT/bitcmp.txt 2>&1 || { rc=1; break; }
done
if [ $rc -eq 0 ]; then
    timeout -k 10 300 python -u tools/sweep_stamps.py --tag=c5lag --n=4096 --T=32 --r=32 --kind=22 > $OUT/stamps.txt 2>&1 &&
    timeout -k 10 600 python -u tools/ab_v3.py $OLD ${MID:+$MID} $NEW --rounds ${ROUNDS:-3} -- \
        --n 4096 --t-per-gpu 32 --latent-dim 32 --steps 10 --warmup 2 --no-secondary > $OUT/ab.txt 2>&1 &&
    timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread -p no:cacheprovider \
        -m gpu tests/test_gpu_w6_workers.py > $OUT/pytest_w6.log 2>&1
    rc=$?
fi
kill $HB
grep -h "EQUAL\|DIFF" $OUT/bitcmp.txt
grep -h "wavefront" $OUT/stamps.txt
grep median $OUT/ab.txt
tail -2 $OUT/pytest_w6.log
exit $rc
