#!/bin/bash
# Odd-width Winograd weight gradient (V = 1 staging): cross-check against the row-window kernel at the
# cnn_deep narrow-block shapes, then the deep fp32 tests and bench line.  Output: gpurun_out/$1/
set -o pipefail
OUT=gpurun_out/${1:-r5ww}
mkdir -p $OUT
for s in "5 25 256 256 24 2 0" "5 25 256 256 23 2 1" "3 13 512 512 17 2 0" "3 13 64 64 9 2 1" "5 25 256 256 4096 5 0" "3 13 512 512 4096 5 0"; do
  timeout -k 5 120 tools/ww_bench $s | tee -a $OUT/ww.txt || { echo "ww_bench $s failed"; exit 1; }
done
timeout -k 10 600 python -u -m pytest tests/test_deep_gpu.py tests/test_fullsize_parity_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread -k "deep" > $OUT/tests.log 2>&1
rc=$?; tail -1 $OUT/tests.log; grep -E "^FAILED" $OUT/tests.log | head -3; [ $rc -eq 0 ] || exit 1
NOTEST=1 DEEP=fp32 bash scripts/r5_deep.sh ${1:-r5ww}
