#!/bin/bash
# 8-wave BN-sum data gradient A/B (PCX_CONVN_EP8=0: the 4-wave instance) on cnn_deep bf16
set -o pipefail
OUT=gpurun_out/${1:-r5ep8}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_deep_bf16_gpu.py tests/test_conv2d_gpu.py -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?; tail -2 $OUT/tests.log; grep -E "^FAILED|Error" $OUT/tests.log | head -5; [ $rc -eq 0 ] || exit 1
for v in 1 0 1 0; do
  PCX_CONVN_EP8=$v timeout -k 10 300 python bench.py --model cnn_deep --precision bf16 --steps 5 --warmup 2 --no-cpu-baseline --no-peaks \
      > $OUT/deep_$v.json 2> $OUT/deep_$v.err || { tail -5 $OUT/deep_$v.err; exit 1; }
  python3 - $OUT/deep_$v.json $v <<'PY'
import json, sys
d = json.load(open(sys.argv[1])); k = d['kernels']
print('ep8', sys.argv[2], d['value'], d['ms_per_step'], {n: round(v['avg_ms'] * v['launches'] / d['steps'], 3) for n, v in k.items() if 'dgrad' in n})
PY
done
echo done
