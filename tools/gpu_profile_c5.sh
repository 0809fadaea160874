#!/bin/bash
# Config 5 per-rank shape (n=4096, T_local=32, r=32: the kind-22 sweep): HBM
# traffic (FETCH_SIZE / WRITE_SIZE passes of their own), SQ counters of the
# sweep, and the rocprofv3 kernel statistics of a bench run.
# usage: tools/gpu_profile_c5.sh TAG [variant]
set -o pipefail
TAG=${1:-c5prof}; VAR=${2:-good}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/$TAG; mkdir -p $OUT
ARGS="--n 4096 --t-per-gpu 32 --latent-dim 32 --variant $VAR --no-cpu-baseline"
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 240 rocprofv3 --pmc $C --kernel-include-regex 'ame_' --output-format csv \
      -d $OUT/pmc_$C -o pmc -- python3 -u bench.py $ARGS --steps 3 --warmup 1 \
      > $OUT/pmc_$C.log 2>&1 || { echo "pmc $C failed"; tail -5 $OUT/pmc_$C.log; exit 1; }
done
python3 tools/pmc_summary.py $OUT n4096_T32_r32_$VAR 4096 32 32 > $OUT/pmc_c5.json || exit 1
cp $OUT/pmc_c5.json profiles/pmc_latest_c5_$VAR.json
cat $OUT/pmc_c5.json
N=4096 TL=32 bash tools/gpu_pmc_sweep.sh $TAG/sq $ARGS || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/stats -o run -- \
    python3 -u bench.py $ARGS --steps 10 --warmup 2 > $OUT/bench.json 2> $OUT/stats.err \
    || { echo "rocprof stats failed"; tail -20 $OUT/stats.err; exit 1; }
cat $OUT/bench.json
find $OUT/stats -name '*kernel_stats.csv'
