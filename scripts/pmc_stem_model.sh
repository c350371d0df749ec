#!/bin/bash
# PMC passes over the cnn_deep bf16 step (stem kernels in their in-model setting)
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/pmcsm
mkdir -p $OUT
ROOT=$(pwd)
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU GRBM_GUI_ACTIVE -f csv -d $ROOT/$OUT/p1 -o run -- python3 $ROOT/bench.py --model cnn_deep --precision bf16 --steps 1 --warmup 1 --no-cpu-baseline --no-peaks --no-kernel-timing > $OUT/p1.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum TCC_EA0_RDREQ_sum TCC_HIT_sum -f csv -d $ROOT/$OUT/p2 -o run -- python3 $ROOT/bench.py --model cnn_deep --precision bf16 --steps 1 --warmup 1 --no-cpu-baseline --no-peaks --no-kernel-timing > $OUT/p2.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --kernel-trace --stats -f csv -d $ROOT/$OUT/kt -o run -- python3 $ROOT/bench.py --model cnn_deep --precision bf16 --steps 3 --warmup 1 --no-cpu-baseline --no-peaks --no-kernel-timing > $OUT/kt.log 2>&1 || exit 1
echo done
