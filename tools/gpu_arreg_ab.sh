#!/bin/bash
# v3 sweep: HF1's AR coefficients held in registers (AME_S3_ARREG=1: both
# halves, =2: Qinv Phi only) instead of read from LDS every step.  Same products
# in the same order, so the fit must be bit-equal to the LDS build; then a
# same-box A/B at config 3 (variant builds s3a0 / s3a1 / s3a2, r = 16).
#   bash tools/gpu_arreg_ab.sh TAG
set -o pipefail
TAG=${1:-arreg}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export PYTHONUNBUFFERED=1
( while sleep 50; do date > $OUT/heartbeat; done ) &
HB=$!
rc=0
for var in good bad naive; do
    for v in 0 1 2; do
        AME_LIB_PATH=tools/_lib/libame_amd_s3a$v.so timeout -k 10 300 python -u tools/bitcmp.py save \
            $OUT/$var$v.npz 1024,16,16 $var 3 3 >> $OUT/bitcmp.txt 2>&1 || { rc=$?; break 2; }
    done
    for v in 1 2; do
        python tools/bitcmp.py cmp $OUT/${var}0.npz $OUT/$var$v.npz >> $OUT/bitcmp.txt 2>&1 || rc=1
    done
done
if [ $rc -eq 0 ]; then
    timeout -k 10 900 python -u tools/ab_v3.py tools/_lib/libame_amd_s3a0.so tools/_lib/libame_amd_s3a1.so \
        tools/_lib/libame_amd_s3a2.so --rounds 5 -- --steps 30 --warmup 3 > $OUT/ab_c3.txt 2>&1
    rc=$?
fi
kill $HB
cat $OUT/bitcmp.txt | grep -E "EQUAL|DIFF|kind"
grep median $OUT/ab_c3.txt
exit $rc
