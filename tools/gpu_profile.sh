#!/bin/bash
# Round profile on the GPU box: HBM traffic of the dominant kernel (two PMC
# passes, FETCH_SIZE and WRITE_SIZE in runs of their own), the bench line
# (CPU baseline included; it reads the PMC result), and the rocprofv3 kernel
# statistics of the same command.  usage: tools/gpu_profile.sh TAG
set -o pipefail
TAG=${1:-prof}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/$TAG; mkdir -p $OUT
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 240 rocprofv3 --pmc $C --kernel-include-regex ame_sweep3_kernel --output-format csv \
      -d $OUT/pmc_$C -o pmc -- python3 -u bench.py --no-cpu-baseline --steps 3 --warmup 1 \
      > $OUT/pmc_$C.log 2>&1 || { echo "pmc $C failed"; tail -5 $OUT/pmc_$C.log; exit 1; }
done
python3 tools/pmc_summary.py $OUT n1024_T128_r16_good > $OUT/pmc_latest.json || exit 1
cp $OUT/pmc_latest.json profiles/pmc_latest.json
cat $OUT/pmc_latest.json
timeout -k 10 400 python3 -u bench.py > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed"; tail -20 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/stats -o run -- \
    python3 -u bench.py --no-cpu-baseline > $OUT/stats_bench.json 2> $OUT/stats.err \
    || { echo "rocprof stats failed"; tail -20 $OUT/stats.err; exit 1; }
find $OUT/stats -name '*kernel_stats.csv'
