#!/bin/bash
# MFMA utilisation per plan label at the headline batch: a kernel trace with the plan's
# ROCTx labels, then two --pmc passes (each <= 8 SQ counters + GRBM_GUI_ACTIVE, no tracing domains) of the
# same bench command, mapped dispatch by dispatch (scripts/pmc_summary.py --label-stalls):
#   pass a: SQ_VALU_MFMA_BUSY_CYCLES, SQ_INSTS_VALU_MFMA_MOPS_F32 / _BF16 (executed MFMA FLOPs / 512), wave
#           cycles, waits, VALU / MFMA instruction counts
#   pass b: LDS / SALU / VMEM instruction counts and their stall cycles
# usage: scripts/pmc_busy4096.sh <out dir> <key> <bench.py args...>
set -eo pipefail
export TMPDIR=/tmp
OUT=$1; KEY=$2; shift 2
ROOT=$(pwd)
mkdir -p "$OUT"
ARGS="--steps 2 --warmup 1 --no-cpu-baseline --no-kernel-timing --no-peaks $*"
PCX_ROCTX=1 timeout -k 10 300 rocprofv3 --kernel-trace --marker-trace --kernel-rename -f csv -d "$ROOT/$OUT/names" -o run -- \
    python3 "$ROOT/bench.py" $ARGS > "$ROOT/$OUT/names.json" 2> "$ROOT/$OUT/names.err"
timeout -s KILL 240 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_F32 SQ_INSTS_VALU_MFMA_MOPS_BF16 \
    SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA GRBM_GUI_ACTIVE \
    -f csv -d "$ROOT/$OUT/pmc_a" -o run -- python3 "$ROOT/bench.py" $ARGS > /dev/null 2> "$ROOT/$OUT/pmc_a.err"
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_LDS \
    SQ_INSTS_SALU SQ_INSTS_VMEM SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE \
    -f csv -d "$ROOT/$OUT/pmc_b" -o run -- python3 "$ROOT/bench.py" $ARGS > /dev/null 2> "$ROOT/$OUT/pmc_b.err"
python3 "$ROOT/scripts/pmc_summary.py" --label-stalls "$ROOT/$OUT/names/run_kernel_trace.csv" \
    "$ROOT/$OUT/pmc_a/run_counter_collection.csv" "$ROOT/gpurun_out/mfma_busy4096.json" "$KEY" > "$ROOT/$OUT/summary_a.txt"
python3 "$ROOT/scripts/pmc_summary.py" --label-stalls "$ROOT/$OUT/names/run_kernel_trace.csv" \
    "$ROOT/$OUT/pmc_b/run_counter_collection.csv" "$ROOT/gpurun_out/mfma_issue4096.json" "$KEY" > "$ROOT/$OUT/summary_b.txt"
echo "pmc-busy4096-done $KEY"
