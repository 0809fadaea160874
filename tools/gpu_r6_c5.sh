#!/bin/bash
# Round 6 config-5 evidence: kind-22 PMC / SQ / rocprof stats at the rank shape,
# then BASELINE config 5's own workload three-way (--config5-full).
set -o pipefail
TAG=${1:-r6c5}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/$TAG; mkdir -p $OUT
bash tools/gpu_profile_c5.sh $TAG || exit 1
timeout -k 10 600 python3 -u bench.py --config5-full > $OUT/config5_full.json 2> $OUT/config5_full.err \
   || { echo "config5 full failed"; tail -20 $OUT/config5_full.err; exit 1; }
cat $OUT/config5_full.json
