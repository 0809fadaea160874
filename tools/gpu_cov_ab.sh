#!/bin/bash
# Covariance-terms kernel (K2): parity of both forms, then same-box A/B of the
# column-per-lane form vs the MFMA form (tools/cov_ab.py).  Variant libraries
# from tools/build_variant.py: c32old / c24old (r = 32 / 24 without the MFMA
# form), c16new / c8new (r = 16 / 8 with it).
#   bash tools/gpu_cov_ab.sh TAG
set -o pipefail
TAG=${1:-cov}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export PYTHONUNBUFFERED=1
PT="python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider"
timeout -k 10 600 $PT -m gpu tests/test_gpu_cov_terms.py > $OUT/pytest_product.log 2>&1 &&
AME_LIB_PATH=tools/_lib/libame_amd_c16new.so timeout -k 10 300 $PT -m gpu tests/test_gpu_cov_terms.py \
    -k "random_spd and -16] or indefinite[16]" > $OUT/pytest_c16new.log 2>&1 &&
AME_LIB_PATH=tools/_lib/libame_amd_c8new.so timeout -k 10 300 $PT -m gpu tests/test_gpu_cov_terms.py \
    -k "random_spd and -8]" > $OUT/pytest_c8new.log 2>&1 &&
L=python-temporal-ame-svi_amd/ame_amd/libame_amd.so &&
timeout -k 10 300 python -u tools/cov_ab.py $L tools/_lib/libame_amd_c32old.so --shapes 4096,32,32 --rounds 3 > $OUT/ab_r32.txt 2>&1 &&
timeout -k 10 300 python -u tools/cov_ab.py $L tools/_lib/libame_amd_c24old.so --shapes 2048,32,24 --rounds 3 > $OUT/ab_r24.txt 2>&1 &&
timeout -k 10 300 python -u tools/cov_ab.py $L tools/_lib/libame_amd_c16new.so --shapes 1024,128,16 --rounds 3 > $OUT/ab_r16.txt 2>&1 &&
timeout -k 10 300 python -u tools/cov_ab.py $L tools/_lib/libame_amd_c8new.so --shapes 256,64,8 --rounds 3 > $OUT/ab_r8.txt 2>&1
rc=$?
tail -3 $OUT/pytest_product.log
cat $OUT/ab_*.txt 2>/dev/null | grep median
exit $rc
