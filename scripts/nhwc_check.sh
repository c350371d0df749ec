#!/bin/bash
# round-4: to_nhwc steps of several image rows for narrow images -- bf16 deep GPU tests and a same-box
# deep bf16 A/B (PCX_NHWC_ROWS1=1 = one row per step)
set -o pipefail
OUT=gpurun_out/nhwc; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "deep or config5 or conv2d" > $OUT/deep_tests.log 2>&1 || { tail -40 $OUT/deep_tests.log; exit 1; }
tail -1 $OUT/deep_tests.log
BENCH_ARGS="--model cnn_deep --precision bf16 --steps 5 --warmup 2" NK=24 ROUNDS=2 timeout -k 10 500 scripts/ab_bench.sh $OUT/ab PCX_NHWC_ROWS1=1:
