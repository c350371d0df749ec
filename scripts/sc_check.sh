#!/bin/bash
# round-4: the stride-2 shortcut data gradient skips its untouched parity classes -- deep GPU tests and
# same-box deep A/Bs against the previous library (variants/prevsc)
set -o pipefail
OUT=gpurun_out/sc; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "deep or fullsize or config5 or conv2d" > $OUT/deep_tests.log 2>&1 || { tail -40 $OUT/deep_tests.log; exit 1; }
tail -1 $OUT/deep_tests.log
BENCH_ARGS="--model cnn_deep --steps 5 --warmup 2" NK=4 ROUNDS=2 timeout -k 10 500 scripts/ab_bench.sh $OUT/ab32 variants/prevsc || exit 1
BENCH_ARGS="--model cnn_deep --precision bf16 --steps 5 --warmup 2" NK=4 ROUNDS=1 timeout -k 10 300 scripts/ab_bench.sh $OUT/ab16 variants/prevsc
