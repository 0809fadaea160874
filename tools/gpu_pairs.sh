#!/bin/bash
# ELBO pair kernel v2 (LDS-DMA) vs v1: parity, isolated kernel statistics of
# both, and the HBM read bytes of v2 (FETCH_SIZE, its own pass).
set -o pipefail
OUT=gpurun_out/${1:-pairs}; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 600 python -u -m pytest tests/test_gpu_pairs.py tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread \
   > $OUT/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
for V in 1 0; do
  AME_PAIRS_V1=$V timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/stats_v1$V -o run -- \
      python3 -u tools/elbo_iso.py > $OUT/iso_v1$V.txt 2> $OUT/iso_v1$V.err || { echo "iso failed"; tail -20 $OUT/iso_v1$V.err; exit 1; }
  F=$(find $OUT/stats_v1$V -name '*kernel_stats.csv' | head -1); cp $F $OUT/kernel_stats_v1$V.csv
  echo "AME_PAIRS_V1=$V"; cat $OUT/iso_v1$V.txt
  python3 -c "
import csv
for r in csv.DictReader(open('$OUT/kernel_stats_v1$V.csv')):
    if 'ame_' in r['Name']: print(r['Name'][:50], r['Calls'], round(float(r['AverageNs'])/1e3,1), 'us', 'min', round(float(r['MinNs'])/1e3,1))"
done
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex ame_pairs --output-format csv \
    -d $OUT/pmc -o pmc -- python3 -u tools/elbo_iso.py --reps 3 > $OUT/pmc.log 2>&1 || { echo "pmc failed"; tail -5 $OUT/pmc.log; exit 1; }
python3 -c "
import csv, glob
v = [float(r['Counter_Value']) for f in glob.glob('$OUT/pmc/**/*counter_collection.csv', recursive=True) for r in csv.DictReader(open(f)) if r['Counter_Name'] == 'FETCH_SIZE']
v = sorted(v); m = v[len(v)//2] * 1024 * 2   # KiB, x2 on gfx950 (MI355X_MICROARCH.md)
print('pair kernel v2 HBM read bytes per launch', m, 'vs algorithmic 536346624 ->', round(m / 536346624, 3))"
