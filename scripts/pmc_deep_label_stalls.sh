#!/bin/bash
# Wait / issue counters per plan label for a cnn_deep bench line (run on the GPU box from the repo root):
# a kernel trace with the plan's ROCTx labels (kernel rename), then ONE --pmc pass of 7 SQ counters +
# GRBM_GUI_ACTIVE (no tracing domains in the counter pass), mapped dispatch by dispatch.
# usage: scripts/pmc_deep_label_stalls.sh <out dir> <key, e.g. cnn_deep/bf16> <bench.py args...>
set -eo pipefail
export TMPDIR=/tmp
OUT=$1; KEY=$2; shift 2
ROOT=$(pwd)
mkdir -p "$OUT"
ARGS="--steps 2 --warmup 1 --no-cpu-baseline --no-kernel-timing --no-peaks $*"
PCX_ROCTX=1 timeout -k 10 300 rocprofv3 --kernel-trace --marker-trace --kernel-rename -f csv -d "$ROOT/$OUT/names" -o run -- \
    python3 "$ROOT/bench.py" $ARGS > "$ROOT/$OUT/names.json" 2> "$ROOT/$OUT/names.err"
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS \
    SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE -f csv -d "$ROOT/$OUT/pmc_stall" -o run -- \
    python3 "$ROOT/bench.py" $ARGS > /dev/null 2> "$ROOT/$OUT/pmc_stall.err"
python3 "$ROOT/scripts/pmc_summary.py" --label-stalls "$ROOT/$OUT/names/run_kernel_trace.csv" \
    "$ROOT/$OUT/pmc_stall/run_counter_collection.csv" "$ROOT/gpurun_out/deep_label_stalls.json" "$KEY" > "$ROOT/$OUT/summary.txt"
echo "label-stalls-done $KEY"
