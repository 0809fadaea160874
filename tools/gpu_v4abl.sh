#!/bin/bash
# v4 ablation timelines: stamped builds with phases removed (timing only, results wrong).
set -o pipefail
OUT=gpurun_out/${1:-v4abl}; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
for T in "" _ng _nw _nc _none; do
  timeout -k 10 200 python -u tools/sweep4_stamps.py --tag=$T > $OUT/stamps$T.txt 2>&1 || { echo "stamps $T failed"; tail -20 $OUT/stamps$T.txt; exit 1; }
  echo "== $T"; grep -A1 "step period" $OUT/stamps$T.txt | head -1
done
