#!/bin/bash
# One rocprofv3 PMC pass of stall / utilisation counters over a short bench run (analysis aid;
# counters only, no tracing domains).  Output: $OUT/pmc_stall/run_counter_collection.csv
set -eo pipefail
export TMPDIR=/tmp
OUT=${1:-gpurun_out/prof_stall}
ROOT=$(pwd)
mkdir -p "$OUT"
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY \
    SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE \
    -f csv -d "$ROOT/$OUT/pmc_stall" -o run -- \
    python3 "$ROOT/bench.py" --steps 2 --warmup 1 --no-cpu-baseline --no-kernel-timing \
    > /dev/null 2> "$ROOT/$OUT/pmc_stall.err"
