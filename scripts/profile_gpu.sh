#!/bin/bash
# rocprofv3 evidence for the bench workload (run on the GPU box from the repo root):
#   1) kernel trace + stats (per-kernel durations)
#   2) separate PMC passes for FETCH_SIZE and WRITE_SIZE (gfx950: FETCH_SIZE counts half the bytes
#      of wide coalesced reads -> doubled in scripts/pmc_summary.py; never combined with tracing)
set -eo pipefail
export TMPDIR=/tmp
OUT=${1:-gpurun_out/prof}
STEPS=${STEPS:-5}
mkdir -p "$OUT"
ROOT=$(pwd)
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d "$ROOT/$OUT/trace" -o run -- \
    python3 "$ROOT/bench.py" --steps "$STEPS" --warmup 2 --no-cpu-baseline --no-kernel-timing \
    > "$ROOT/$OUT/bench_trace.json" 2> "$ROOT/$OUT/bench_trace.err"
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -f csv -d "$ROOT/$OUT/pmc_fetch" -o run -- \
    python3 "$ROOT/bench.py" --steps 2 --warmup 1 --no-cpu-baseline --no-kernel-timing \
    > /dev/null 2> "$ROOT/$OUT/pmc_fetch.err"
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -f csv -d "$ROOT/$OUT/pmc_write" -o run -- \
    python3 "$ROOT/bench.py" --steps 2 --warmup 1 --no-cpu-baseline --no-kernel-timing \
    > /dev/null 2> "$ROOT/$OUT/pmc_write.err"
python3 "$ROOT/scripts/pmc_summary.py" "$OUT" "$ROOT/$OUT/pmc_traffic.json" "$ROOT/$OUT/trace_layers.json" > /dev/null
