#!/bin/bash
# Winograd weight gradient (wgrad_wino) vs the pixel-stream kernel (wgrad_s) on the cnn_small layer
# shapes (B = 4096) and a few ragged ones: times, dW relative difference, dy difference.
set -o pipefail
cd "$(dirname "$0")"
for s in "40 200 32 32 4096 5 1" "20 100 32 64 4096 5 0" "20 100 64 64 4096 5 1" "10 50 64 128 4096 5 0" \
         "10 50 128 128 4096 5 1" "9 28 32 64 37 3 1" "7 14 64 32 5 3 0" "11 16 32 32 3 3 1" ${EXTRA}; do
  timeout -k 5 60 ./ww_bench $s || exit 1
done
