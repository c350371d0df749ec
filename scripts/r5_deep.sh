#!/bin/bash
# cnn_deep iteration on the GPU box (repo root): bf16 / conv tests, then the deep bench lines.
# Output under gpurun_out/$1.  Stops at the first failing step.
set -o pipefail
OUT=gpurun_out/${1:-r5deep}
mkdir -p $OUT
export TMPDIR=/tmp
if [ -z "$NOTEST" ]; then
  timeout -k 10 600 python -u -m pytest ${TESTS:-tests/test_deep_bf16_gpu.py tests/test_conv2d_gpu.py tests/test_config5_gpu.py tests/test_stem_fused_gpu.py} \
      -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1
  rc=$?; tail -2 $OUT/tests.log; grep -E "^FAILED|Error" $OUT/tests.log | head -5; [ $rc -eq 0 ] || exit 1
fi
for m in ${DEEP:-bf16}; do
  timeout -k 10 300 python bench.py --model cnn_deep --precision $m --steps 5 --warmup 2 --no-cpu-baseline --no-peaks \
      > $OUT/deep_$m.json 2> $OUT/deep_$m.err || { tail -5 $OUT/deep_$m.err; exit 1; }
  python3 - $OUT/deep_$m.json $m <<'PY'
import json, sys, re, collections
d = json.load(open(sys.argv[1])); r = d['roofline']
print('deep', sys.argv[2], d['value'], d['ms_per_step'], r['kernel'], r['frac'], d['step_roofline']['mfma_fraction'])
k = d['kernels']
print(sorted(((round(v['avg_ms'] * v['launches'] / d['steps'], 3), n, v.get('exec_frac')) for n, v in k.items()), reverse=True)[:24])
PY
done
echo r5-deep-done
