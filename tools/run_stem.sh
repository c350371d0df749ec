#!/bin/bash
# Fused bf16 stem (y0 recomputed) vs the kernels that keep y0: bit-exactness and times at the
# cnn_deep T = 200 shape (B = 4096) and at ragged shapes (odd H, W % 4 != 0, partial column blocks).
set -o pipefail
cd "$(dirname "$0")"
for s in "4096 40 200 5" "37 9 30 2" "5 13 57 2" "3 40 256 2" ${EXTRA}; do
  timeout -k 5 90 ./stem_bench $s || exit 1
done
