#!/bin/bash
# v3 stamp timelines of ablated builds (timing only; the results are wrong by design).
set -o pipefail
OUT=gpurun_out/${1:-v3abl}; shift; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
for T in "$@"; do
  timeout -k 10 200 python -u tools/sweep3_stamps.py --tag=$T > $OUT/stamps$T.txt 2>&1 || { echo "stamps $T failed"; tail -20 $OUT/stamps$T.txt; exit 1; }
  echo "== $T"; grep "step period" $OUT/stamps$T.txt; grep -E "^\s+[0-9]+ " $OUT/stamps$T.txt | tr -s ' ' | paste -sd' '
done
