#!/bin/bash
# round-4: stem forward kernels at 3-4 waves per SIMD -- deep GPU tests and same-box deep A/Bs against the
# previous library (variants/prevstem)
set -o pipefail
OUT=gpurun_out/stemocc; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "deep or fullsize or stem" > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
BENCH_ARGS="--model cnn_deep --steps 5 --warmup 2" NK=40 ROUNDS=1 timeout -k 10 300 scripts/ab_bench.sh $OUT/ab32 variants/prevstem || exit 1
BENCH_ARGS="--model cnn_deep --precision bf16 --steps 5 --warmup 2" NK=40 ROUNDS=1 timeout -k 10 300 scripts/ab_bench.sh $OUT/ab16 variants/prevstem
