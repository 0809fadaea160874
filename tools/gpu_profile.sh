#!/bin/bash
# Round profile on the GPU box: HBM traffic of the sweep / pair / covariance
# kernels (two PMC passes, FETCH_SIZE and WRITE_SIZE in runs of their own),
# MFMA busy of the pair kernel, the bench line (CPU baseline included; it reads
# the PMC result), and the rocprofv3 kernel statistics of the same command.
# usage: tools/gpu_profile.sh TAG
set -o pipefail
TAG=${1:-prof}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/$TAG; mkdir -p $OUT
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 240 rocprofv3 --pmc $C --kernel-include-regex 'ame_' --output-format csv \
      -d $OUT/pmc_$C -o pmc -- python3 -u bench.py --no-cpu-baseline --steps 3 --warmup 1 \
      > $OUT/pmc_$C.log 2>&1 || { echo "pmc $C failed"; tail -5 $OUT/pmc_$C.log; exit 1; }
done
timeout -s KILL 240 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-include-regex ame_pairs \
    --output-format csv -d $OUT/pmc_pairs_mfma -o pmc -- python3 -u bench.py --no-cpu-baseline --steps 3 --warmup 1 \
    > $OUT/pmc_pairs_mfma.log 2>&1 || { echo "pmc pairs mfma failed"; tail -5 $OUT/pmc_pairs_mfma.log; exit 1; }
python3 tools/pmc_pairs.py $OUT > $OUT/pmc_pairs.json || exit 1
cat $OUT/pmc_pairs.json
python3 tools/pmc_summary.py $OUT n1024_T128_r16_good 1024 128 16 > $OUT/pmc_latest.json || exit 1
cp $OUT/pmc_latest.json profiles/pmc_latest.json
cat $OUT/pmc_latest.json
# SQ counters of the sweep (in-order sweeps: no pipelined launch waits in the counts)
bash tools/gpu_pmc_sweep.sh $TAG/sq --no-pipeline || exit 1
timeout -k 10 400 python3 -u bench.py > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed"; tail -20 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/stats -o run -- \
    python3 -u bench.py --no-cpu-baseline > $OUT/stats_bench.json 2> $OUT/stats.err \
    || { echo "rocprof stats failed"; tail -20 $OUT/stats.err; exit 1; }
find $OUT/stats -name '*kernel_stats.csv'
