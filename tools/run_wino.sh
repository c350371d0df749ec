#!/bin/bash
# Winograd conv vs direct LDS-DMA conv on the cnn_small layer shapes (B = 4096), all epilogues used
set -o pipefail
cd "$(dirname "$0")"
for s in "40 200 32 32 4096 5 0 1" "40 200 32 32 4096 5 1 0" "20 100 32 64 4096 5 0 0" "20 100 64 32 4096 5 2 0" \
         "20 100 64 64 4096 5 0 1" "20 100 64 64 4096 5 1 0" "10 50 64 128 4096 5 0 0" "10 50 128 64 4096 5 2 0" \
         "10 50 128 128 4096 5 0 1" "10 50 128 128 4096 5 1 0" "40 201 32 32 512 3 0 1" "40 201 32 32 512 3 1 0" \
         "20 100 64 32 512 3 2 0" "20 100 64 64 512 3 3 0" ${EXTRA}; do
  timeout -k 5 60 ./wino_bench $s || exit 1
done
