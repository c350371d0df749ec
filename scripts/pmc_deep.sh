#!/bin/bash
# rocprofv3 HBM traffic per plan label for a bench workload (run on the GPU box from the repo root):
#   1) kernel trace of the command with PCX_ROCTX=1 under --marker-trace --kernel-rename: every
#      dispatch named by the plan's profiler label
#   2) separate --pmc passes for FETCH_SIZE and WRITE_SIZE of the same command (no tracing domains)
#   3) scripts/pmc_summary.py --labels: dispatch k of the PMC passes carries label k of the trace
# usage: scripts/pmc_deep.sh <out dir> <key, e.g. cnn_deep/bf16> <bench.py args...>
set -eo pipefail
export TMPDIR=/tmp
OUT=$1; KEY=$2; shift 2
ROOT=$(pwd)
mkdir -p "$OUT"
ARGS="--steps 2 --warmup 1 --no-cpu-baseline --no-kernel-timing --no-peaks $*"
PCX_ROCTX=1 timeout -k 10 300 rocprofv3 --kernel-trace --marker-trace --kernel-rename -f csv -d "$ROOT/$OUT/names" -o run -- \
    python3 "$ROOT/bench.py" $ARGS > "$ROOT/$OUT/names.json" 2> "$ROOT/$OUT/names.err"
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -f csv -d "$ROOT/$OUT/pmc_fetch" -o run -- \
    python3 "$ROOT/bench.py" $ARGS > /dev/null 2> "$ROOT/$OUT/pmc_fetch.err"
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -f csv -d "$ROOT/$OUT/pmc_write" -o run -- \
    python3 "$ROOT/bench.py" $ARGS > /dev/null 2> "$ROOT/$OUT/pmc_write.err"
python3 "$ROOT/scripts/pmc_summary.py" --labels "$ROOT/$OUT/names/run_kernel_trace.csv" "$OUT" \
    "$ROOT/$OUT/pmc_traffic.json" "$KEY" > "$ROOT/$OUT/summary.txt"
echo "pmc-labels-done $KEY"
