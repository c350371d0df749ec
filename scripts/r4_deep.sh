#!/bin/bash
# Round-4 deep check on the GPU box (repo root): the cnn_deep GPU tests, then the bf16 (and optionally
# fp32) bench lines.  Output under gpurun_out/$1.
set -o pipefail
OUT=gpurun_out/${1:-r4deep}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "deep or config5 or conv2d" > $OUT/gpu_tests.log 2>&1
rc=$?; tail -2 $OUT/gpu_tests.log; grep -E "^FAILED|Error" $OUT/gpu_tests.log | head -5; [ $rc -eq 0 ] || exit 1
for m in ${DEEP:-bf16}; do
  timeout -k 10 300 python bench.py --model cnn_deep --precision $m --steps 5 --warmup 2 --no-cpu-baseline --no-peaks \
      > $OUT/deep_$m.json 2> $OUT/deep_$m.err || { tail -5 $OUT/deep_$m.err; exit 1; }
  python3 -c "import json;d=json.load(open('$OUT/deep_$m.json'));print('deep $m', d['value'], d['ms_per_step'], d['roofline']['kernel'], d['roofline']['frac']); k=d['kernels']; print({n: k[n]['avg_ms'] for n in list(k)[:14]})"
done
echo r4-deep-done
