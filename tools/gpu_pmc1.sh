#!/bin/bash
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
OUT=gpurun_out/pmc1; mkdir -p $OUT
timeout -s KILL 60 rocprofv3 -L > $OUT/avail.txt 2>&1; echo "list rc=$?"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT --kernel-include-regex sweep3_kernel --output-format csv -d $OUT/p1 -o p1 -- python3 -u bench.py --no-cpu-baseline --steps 2 --warmup 0 > $OUT/p1.log 2>&1
echo "pass1 rc=$?"; ls $OUT/p1 2>/dev/null | head
