#!/bin/bash
# Kind-22 workgroup entry / slice start stamps at config 5's rank shape, two runs.
#   bash tools/gpu_c5_entry.sh TAG
set -o pipefail
TAG=${1:-c5entry}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u tools/sweep_stamps.py --tag=c5lag --n=4096 --T=32 --r=32 --kind=22 > $OUT/run1.txt 2>&1 &&
timeout -k 10 300 python -u tools/sweep_stamps.py --tag=c5lag --n=4096 --T=32 --r=32 --kind=22 > $OUT/run2.txt 2>&1
rc=$?
grep -h "wavefront\|latest" $OUT/run1.txt $OUT/run2.txt
exit $rc
