#!/bin/bash
# Round 6 (session 2): parity subset, then same-box timing of the in-tree library against variant builds on the
# cnn_deep bf16 and fp32 lines (and the cnn_small line).  Usage: scripts/r6s2_deep_ab.sh TAG "pytest selection" dir...
set -o pipefail
OUT=gpurun_out/${1:-r6s2deep}; SEL=$2; shift 2
mkdir -p $OUT
export TMPDIR=/tmp
if [ -n "$SEL" ]; then
  timeout -k 10 700 python -u -m pytest $SEL -m gpu -x -q -s --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1
  rc=$?; grep -E "passed|failed" $OUT/gpu_tests.log | tail -2; grep -E "^FAILED|Error" $OUT/gpu_tests.log | head -5; [ $rc -eq 0 ] || exit 1
fi
BENCH_ARGS="--model cnn_deep --precision bf16 --steps 5 --warmup 2" ROUNDS=2 NK=12 bash scripts/ab_bench.sh $OUT/bf16 "$@" || exit 1
BENCH_ARGS="--model cnn_deep --precision fp32 --steps 3 --warmup 1" ROUNDS=1 NK=8 bash scripts/ab_bench.sh $OUT/fp32 "$@" || exit 1
ROUNDS=1 NK=6 bash scripts/ab_bench.sh $OUT/small "$@" || exit 1
