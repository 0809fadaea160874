#!/bin/bash
# SQ / SQC counters of the sweep kernel, v4 and v3, one --pmc pass per counter group.
set -o pipefail
OUT=gpurun_out/${1:-pmcsq}; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
PA="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_WAIT_INST_LDS"
PB="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_INSTS_MFMA SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_IFETCH"
PC="SQC_ICACHE_MISSES SQC_ICACHE_HITS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE"
for V in 4 3; do
  for P in A B C; do
    eval CN=\$P$P
    if [[ $V == 4 ]]; then export AME_SWEEP_V4=1; else unset AME_SWEEP_V4; fi
    timeout -s KILL 90 rocprofv3 --pmc $CN --kernel-include-regex ame_sweep --output-format csv \
      -d $OUT/v$V/p$P -o pmc -- python3 -u bench.py --no-cpu-baseline --steps 3 --warmup 1 \
      > $OUT/v${V}_p$P.log 2>&1 || { echo "pmc v$V $P failed"; tail -5 $OUT/v${V}_p$P.log; exit 1; }
  done
  echo "=== v$V"; python3 tools/pmc_sq.py $OUT/v$V 1024 128 | tee $OUT/v$V.txt
done
