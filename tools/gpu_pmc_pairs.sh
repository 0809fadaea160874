#!/bin/bash
# SQ counters of the isolated ELBO pair kernel, v1 and v2 (one --pmc pass per group).
set -o pipefail
OUT=gpurun_out/${1:-pmcpairs}; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
PA="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_WAIT_INST_LDS"
PB="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_INSTS_MFMA SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_IFETCH"
PC="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE"
for V in 1 0; do
  for P in A B C; do
    eval CN=\$P$P
    AME_PAIRS_V1=$V timeout -s KILL 90 rocprofv3 --pmc $CN --kernel-include-regex ame_pairs --output-format csv \
      -d $OUT/v1$V/p$P -o pmc -- python3 -u tools/elbo_iso.py --reps 3 \
      > $OUT/v1${V}_p$P.log 2>&1 || { echo "pmc v1=$V $P failed"; tail -5 $OUT/v1${V}_p$P.log; exit 1; }
  done
  echo "=== AME_PAIRS_V1=$V"; python3 tools/pmc_sq.py $OUT/v1$V 1024 128 ame_pairs | tee $OUT/v1$V.txt
done
