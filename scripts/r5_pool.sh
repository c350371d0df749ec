#!/bin/bash
# bn_relu_pool: NI quads per thread per pass (PCX_POOL_NI=1: the previous one-quad loop), cnn_small A/B
set -o pipefail
OUT=gpurun_out/${1:-r5pool}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest ${TESTS:-tests/test_model_gpu.py tests/test_small_shapes_gpu.py tests/test_fullsize_parity_gpu.py} -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?; tail -2 $OUT/tests.log; grep -E "^FAILED|Error" $OUT/tests.log | head -5; [ $rc -eq 0 ] || exit 1
for v in 2 1 2 1; do
  PCX_POOL_NI=$v timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-peaks \
      > $OUT/small_$v.json 2> $OUT/small_$v.err || { tail -5 $OUT/small_$v.err; exit 1; }
  python3 - $OUT/small_$v.json $v <<'PY'
import json, sys
d = json.load(open(sys.argv[1])); k = d['kernels']
print('ni', sys.argv[2], d['value'], d['ms_per_step'], {n: round(v['avg_ms'], 3) for n, v in k.items() if 'pool' in n})
PY
done
echo done
