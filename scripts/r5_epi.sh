#!/bin/bash
# Winograd engines' cross-checks and timings on the cnn_small layer shapes (GPU box, repo root): conv_wino vs
# the direct conv for every epilogue.  Output: gpurun_out/$1/epi.txt
set -o pipefail
OUT=gpurun_out/${1:-r5epi}
mkdir -p $OUT
for s in "40 200 32 32 4096 5 0 1" "20 100 64 64 4096 5 0 1" "20 100 32 64 4096 5 0 0" "10 50 128 128 4096 5 0 1" \
         "10 50 64 128 4096 5 0 0" "20 100 64 64 4096 5 1 0" "10 50 128 128 4096 5 1 0" "20 100 64 32 4096 5 4 0" \
         "10 50 128 64 4096 5 4 0" "20 100 64 32 512 3 2 0" "20 100 64 64 512 3 3 0" "21 101 32 32 64 3 0 1" \
         "21 101 32 32 64 3 1 0" "21 101 32 32 64 3 3 0" "10 50 128 128 24 5 0 1"; do
  timeout -k 5 60 tools/wino_bench $s | tee -a $OUT/epi.txt || { echo "wino_bench $s failed"; exit 1; }
done
echo epi-done
