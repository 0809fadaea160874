#!/bin/bash
# Isolated ELBO kernel statistics for the default library and variant libraries
# (tools/interference.py --build TAG DEFS); usage: gpu_pairs_var.sh OUT TAG...
set -o pipefail
OUT=gpurun_out/${1:-pvar}; mkdir -p $OUT; shift
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
B=python-temporal-ame-svi_amd/ame_amd/_build
for T in default "$@"; do
  if [[ $T == default ]]; then unset AME_LIB_PATH; else export AME_LIB_PATH=$B/libame_amd_var$T.so; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/stats_$T -o run -- \
      python3 -u tools/elbo_iso.py > $OUT/iso_$T.txt 2> $OUT/iso_$T.err || { echo "iso $T failed"; tail -20 $OUT/iso_$T.err; exit 1; }
  F=$(find $OUT/stats_$T -name '*kernel_stats.csv' | head -1)
  echo "== $T"; python3 -c "
import csv
for r in csv.DictReader(open('$F')):
    if 'ame_pairs' in r['Name'] or 'ame_nodes' in r['Name'] or 'ame_cov' in r['Name']: print(r['Name'][:40], r['Calls'], round(float(r['AverageNs'])/1e3,1), 'us', 'min', round(float(r['MinNs'])/1e3,1))"
done
