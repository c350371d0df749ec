#!/bin/bash
# wgrad_s vs round-1 kernels on the cnn_small layer shapes (B = 4096) + a few ragged / deep shapes
set -o pipefail
cd "$(dirname "$0")"
export LD_LIBRARY_PATH=$PWD/../phoneme_contrast_amd:$LD_LIBRARY_PATH
for s in "40 200 32 32 4096 5 1" "20 100 32 64 4096 5 0" "20 100 64 64 4096 5 1" "10 50 64 128 4096 5 0" \
         "10 50 128 128 4096 5 1" "40 201 32 32 512 3 1" "5 25 128 128 4096 5 0" "3 13 256 256 4096 5 0" \
         "2 7 512 512 4096 5 0" ${EXTRA}; do
  timeout -k 5 60 ./ws_bench $s || exit 1
done
