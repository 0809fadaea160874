#!/bin/bash
# Parity subset (all latent dims 1..32 build) + ELBO-side interference diagnostic.
set -o pipefail
OUT=gpurun_out/${1:-r02b}; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_pairs.py tests/test_capi.py -m gpu -x -q --timeout 300 --timeout-method thread \
   > $OUT/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
shift
timeout -k 10 500 python -u tools/interference.py "$@" > $OUT/interference.txt 2>&1 || { echo "interference failed"; tail -20 $OUT/interference.txt; exit 1; }
cat $OUT/interference.txt
