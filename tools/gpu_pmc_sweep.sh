#!/bin/bash
# SQ / SQC counters of the sweep kernel (one --pmc pass per counter group);
# extra arguments go to bench.py (e.g. --n 4096 --t-per-gpu 32 --latent-dim 32);
# N / TL (env, default 1024 / 128) normalise the counters per workgroup-step.
# usage: [N=4096 TL=32] tools/gpu_pmc_sweep.sh TAG [bench args...]
set -o pipefail
OUT=gpurun_out/${1:-pmcsq}; shift; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
PA="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_WAIT_INST_LDS"
PB="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_INSTS_MFMA SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_IFETCH"
PC="SQC_ICACHE_MISSES SQC_ICACHE_HITS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE"
for P in A B C; do
  eval CN=\$P$P
  timeout -s KILL 90 rocprofv3 --pmc $CN --kernel-include-regex ame_sweep --output-format csv \
    -d $OUT/p$P -o pmc -- python3 -u bench.py --no-cpu-baseline --steps 3 --warmup 1 "$@" \
    > $OUT/p$P.log 2>&1 || { echo "pmc $P failed"; tail -5 $OUT/p$P.log; exit 1; }
done
python3 tools/pmc_sq.py $OUT ${N:-1024} ${TL:-128} | tee $OUT/sq.txt
