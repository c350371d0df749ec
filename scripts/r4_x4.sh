#!/bin/bash
# conv_wino 16-byte staging (X4): engine cross-check on every cnn_small shape, X4 vs dword-copy timing at
# B = 4096, then the GPU tests and the bench.  Output under gpurun_out/$1.
set -o pipefail
OUT=gpurun_out/${1:-r4x4}
mkdir -p $OUT
export TMPDIR=/tmp
export PCX_FULLSIZE_JSON=$(pwd)/$OUT/fullsize_parity.json
cd tools
for s in "40 200 32 32 48 1 0 1" "20 100 32 64 48 1 0 0" "40 200 32 32 48 1 1 0" "20 100 64 32 48 1 2 0" "10 50 128 64 48 1 2 0" \
         "40 201 32 32 24 1 0 1" "40 201 32 32 24 1 1 0" "20 100 64 64 24 1 3 0" "10 50 128 128 24 1 0 1" "10 50 128 128 24 1 1 0" \
         "20 101 64 64 16 1 0 1" "20 101 64 64 16 1 1 0"; do
  timeout -k 5 60 ./wino_bench $s >> ../$OUT/x4_check.log 2>&1 || { echo "wino_bench $s failed"; tail -3 ../$OUT/x4_check.log; exit 1; }
done
tail -13 ../$OUT/x4_check.log
for s in "40 200 32 32 4096 5 0 1" "20 100 32 64 4096 5 0 0" "20 100 64 64 4096 5 0 1" "20 100 64 64 4096 5 1 0" \
         "10 50 64 128 4096 5 0 0" "10 50 128 128 4096 5 0 1" "10 50 128 128 4096 5 1 0"; do
  for x in 1 0; do
    PCX_WINO_X4=$x timeout -k 5 60 ./wino_bench $s 2>&1 | sed "s/^/x4=$x /" >> ../$OUT/x4_time.log || exit 1
  done
done
cat ../$OUT/x4_time.log
cd ..
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1
rc=$?; tail -2 $OUT/gpu_tests.log; grep -E "^FAILED|Error" $OUT/gpu_tests.log | head -5; [ $rc -eq 0 ] || exit 1
timeout -k 10 500 python bench.py --cpu-quick > $OUT/bench.json 2> $OUT/bench.err || { tail -5 $OUT/bench.err; exit 1; }
python3 -c "import json;d=json.load(open('$OUT/bench.json'));print('small', d['value'], d['ms_per_step'], d['roofline']['kernel'], d['roofline']['frac']); print({k: v['avg_ms'] for k, v in list(d['kernels'].items())[:16]})"
echo r4-x4-done
