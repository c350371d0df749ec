#!/bin/bash
# round-4: batch-spanning Winograd units for cnn_deep's narrow blocks -- engine cross-checks, the deep
# GPU tests, a same-box deep fp32 A/B (PCX_NO_WINO_SPAN=1 = direct LDS-DMA conv) and timing of the shapes
set -o pipefail
OUT=gpurun_out/span; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_wino_engine_gpu.py -x -q --timeout 120 --timeout-method thread > $OUT/wino_tests.log 2>&1 || { tail -30 $OUT/wino_tests.log; exit 1; }
tail -1 $OUT/wino_tests.log
for s in "5 25 256 256 4096 5 0 0" "5 25 256 256 4096 5 3 0" "3 13 512 512 4096 5 0 0" "3 13 512 512 4096 5 3 0" "5 26 256 256 4096 5 0 0" "3 13 512 512 4096 5 0 0"; do
  WINO_QUEUE=1 timeout -k 5 60 tools/wino_bench $s || exit 1
done > $OUT/shapes.txt 2>&1 || { cat $OUT/shapes.txt; exit 1; }
cat $OUT/shapes.txt
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "deep or fullsize or conv2d" > $OUT/deep_tests.log 2>&1 || { tail -30 $OUT/deep_tests.log; exit 1; }
tail -1 $OUT/deep_tests.log
BENCH_ARGS="--model cnn_deep --steps 5 --warmup 2" NK=12 ROUNDS=2 timeout -k 10 500 scripts/ab_bench.sh $OUT/ab PCX_NO_WINO_SPAN=1:
