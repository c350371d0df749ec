#!/bin/bash
# round-4: channel-last engine occupancy (BN-sum epilogue as its own instantiation, waves_per_eu 2) --
# bf16 GPU tests and a same-box deep bf16 A/B against the previous library (variants/prevcn)
set -o pipefail
OUT=gpurun_out/cn; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "deep or config5 or conv2d" > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
BENCH_ARGS="--model cnn_deep --precision bf16 --steps 5 --warmup 2" NK=30 ROUNDS=2 timeout -k 10 400 scripts/ab_bench.sh $OUT/ab16 variants/prevcn
