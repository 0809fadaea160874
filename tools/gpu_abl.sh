#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/abl
for t in "" nofma nored noprio; do
  timeout -k 10 120 python -u tools/sweep3_stamps.py --tag=$t > gpurun_out/abl/st_$t.txt 2>&1 || exit 1
  echo "== $t"; grep -A8 "step period\|hw0(w1)" gpurun_out/abl/st_$t.txt | head -14
done
