#!/bin/bash
# bf16 conv-output planes A/B (PCX_NO_Y16=1: float32 planes) on cnn_deep bf16
set -o pipefail
OUT=gpurun_out/${1:-r5y16}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -s tests/test_deep_bf16_gpu.py tests/test_conv2d_gpu.py tests/test_config5_gpu.py tests/test_stem_fused_gpu.py -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?; tail -2 $OUT/tests.log; grep -E "^FAILED|Error" $OUT/tests.log | head -5; [ $rc -eq 0 ] || exit 1
for v in 0 1 0 1; do
  PCX_NO_Y16=$v timeout -k 10 300 python bench.py --model cnn_deep --precision bf16 --steps 5 --warmup 2 --no-cpu-baseline --no-peaks \
      > $OUT/deep_$v.json 2> $OUT/deep_$v.err || { tail -5 $OUT/deep_$v.err; exit 1; }
  python3 - $OUT/deep_$v.json $v <<'PY'
import json, sys
d = json.load(open(sys.argv[1])); k = d['kernels']
print('noy16', sys.argv[2], d['value'], d['ms_per_step'], {n: round(v['avg_ms'] * v['launches'] / d['steps'], 3) for n, v in k.items() if n.split('_L')[0] in ('bn_act','dy_nhwc','bwd_prep','conv_fwd','conv_dgrad') and n[-1] in '12'})
PY
done
echo done
