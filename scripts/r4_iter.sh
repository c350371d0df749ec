#!/bin/bash
# Round-4 iteration on the GPU box (repo root): GPU tests, the bench (B = 24 CPU leg only), cnn_deep lines
# on request.  Output under gpurun_out/$1.  Stops at the first failing step.
set -o pipefail
OUT=gpurun_out/${1:-r4it}
mkdir -p $OUT
export TMPDIR=/tmp
export PCX_FULLSIZE_JSON=$(pwd)/$OUT/fullsize_parity.json
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1
rc=$?; tail -2 $OUT/gpu_tests.log; grep -E "^FAILED|Error" $OUT/gpu_tests.log | head -5; [ $rc -eq 0 ] || exit 1
timeout -k 10 500 python bench.py --cpu-quick > $OUT/bench.json 2> $OUT/bench.err || { tail -5 $OUT/bench.err; exit 1; }
python3 -c "import json;d=json.load(open('$OUT/bench.json'));print('small', d['value'], d['ms_per_step'], d['roofline']['kernel'], d['roofline']['frac']); print({k: v['avg_ms'] for k, v in list(d['kernels'].items())[:18]})"
for m in ${DEEP:-}; do
  timeout -k 10 300 python bench.py --model cnn_deep --precision $m --steps 5 --warmup 2 --no-cpu-baseline --no-peaks \
      > $OUT/deep_$m.json 2> $OUT/deep_$m.err || { tail -5 $OUT/deep_$m.err; exit 1; }
  python3 -c "import json;d=json.load(open('$OUT/deep_$m.json'));print('deep $m', d['value'], d['ms_per_step'], d['roofline']['kernel'], d['roofline']['frac'])"
done
echo r4-iter-done
