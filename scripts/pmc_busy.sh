#!/bin/bash
# MFMA-busy / issue counters per plan label at a reduced batch (run on the GPU box from the repo root).
# At B = 4096 the SQ_VALU_MFMA_BUSY_CYCLES sums of the 3-5 ms conv kernels exceed 2^31-2^32 and come
# out saturated (round 3); at B = 512 every launch stays below 2^30 while its grid still covers the chip
# many times over (cnn_small L2: 16384 Winograd units for 512 workgroups).  A kernel trace with the
# plan's ROCTx labels, then ONE --pmc pass (7 SQ counters + GRBM_GUI_ACTIVE, no tracing domains),
# mapped dispatch by dispatch.  usage: scripts/pmc_busy.sh <out dir> <key> <bench.py args...>
set -eo pipefail
export TMPDIR=/tmp
OUT=$1; KEY=$2; shift 2
ROOT=$(pwd)
mkdir -p "$OUT"
ARGS="--steps 2 --warmup 1 --no-cpu-baseline --no-kernel-timing --no-peaks $*"
PCX_ROCTX=1 timeout -k 10 300 rocprofv3 --kernel-trace --marker-trace --kernel-rename -f csv -d "$ROOT/$OUT/names" -o run -- \
    python3 "$ROOT/bench.py" $ARGS > "$ROOT/$OUT/names.json" 2> "$ROOT/$OUT/names.err"
timeout -s KILL 240 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY \
    SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE -f csv -d "$ROOT/$OUT/pmc_busy" -o run -- \
    python3 "$ROOT/bench.py" $ARGS > /dev/null 2> "$ROOT/$OUT/pmc_busy.err"
python3 "$ROOT/scripts/pmc_summary.py" --label-stalls "$ROOT/$OUT/names/run_kernel_trace.csv" \
    "$ROOT/$OUT/pmc_busy/run_counter_collection.csv" "$ROOT/gpurun_out/mfma_busy.json" "$KEY" > "$ROOT/$OUT/summary.txt"
echo "pmc-busy-done $KEY"
