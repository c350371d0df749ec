#!/bin/bash
# round-4 analysis: blocks per channel-reduction launch (chan_slices target 2048 vs 8192 / 16384), deep fp32 / bf16
set -o pipefail
OUT=gpurun_out/chan; mkdir -p $OUT
BENCH_ARGS="--model cnn_deep --steps 5 --warmup 2" NK=3 ROUNDS=2 timeout -k 10 600 scripts/ab_bench.sh $OUT/ab32 PCX_CHAN_TARGET=8192: PCX_CHAN_TARGET=16384: || exit 1
BENCH_ARGS="--model cnn_deep --precision bf16 --steps 5 --warmup 2" NK=3 ROUNDS=1 timeout -k 10 300 scripts/ab_bench.sh $OUT/ab16 PCX_CHAN_TARGET=8192:
