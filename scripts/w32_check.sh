#!/bin/bash
# round-4: wgrad_w32 row stream across tasks -- cross-checks vs the pixel-stream kernel, the deep GPU
# tests, and a same-box deep fp32 A/B against the per-task pipeline (variants/oldw32)
set -o pipefail
OUT=gpurun_out/w32; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_wino_engine_gpu.py -x -q --timeout 120 --timeout-method thread -k row_window > $OUT/ws_tests.log 2>&1 || { tail -30 $OUT/ws_tests.log; exit 1; }
tail -1 $OUT/ws_tests.log
for s in "3 13 512 512 4096 5 0" "5 25 256 256 4096 5 0"; do timeout -k 5 60 tools/ws_bench $s || exit 1; done > $OUT/shapes.txt 2>&1 || { cat $OUT/shapes.txt; exit 1; }
cat $OUT/shapes.txt
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "deep or fullsize" > $OUT/deep_tests.log 2>&1 || { tail -30 $OUT/deep_tests.log; exit 1; }
tail -1 $OUT/deep_tests.log
BENCH_ARGS="--model cnn_deep --steps 5 --warmup 2" NK=12 ROUNDS=2 timeout -k 10 500 scripts/ab_bench.sh $OUT/ab variants/oldw32
