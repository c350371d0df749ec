#!/bin/bash
# One PMC stall / utilisation pass over the cnn_deep bf16 step (analysis aid; counters only)
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/pmcds
mkdir -p $OUT
ROOT=$(pwd)
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAVES GRBM_GUI_ACTIVE -f csv -d $ROOT/$OUT/p1 -o run -- python3 $ROOT/bench.py --model cnn_deep --precision bf16 --steps 1 --warmup 1 --no-cpu-baseline --no-peaks --no-kernel-timing > $OUT/p1.log 2>&1 || exit 1
echo done
