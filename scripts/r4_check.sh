#!/bin/bash
# Round-4 GPU check (repo root): all GPU tests, the default bench line (CPU baseline with the
# B = 4096 leg), the cnn_deep bf16 line.  Output under gpurun_out/$1 (default r4).
set -o pipefail
OUT=gpurun_out/${1:-r4}
mkdir -p $OUT
export TMPDIR=/tmp
export PCX_FULLSIZE_JSON=$(pwd)/$OUT/fullsize_parity.json
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1
rc=$?; tail -3 $OUT/gpu_tests.log; grep -E "FAILED|Error" $OUT/gpu_tests.log | head -5; [ $rc -eq 0 ] || exit 1
timeout -k 10 500 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -5 $OUT/bench.err; exit 1; }
python3 -c "import json;d=json.load(open('$OUT/bench.json'));print('small', d['value'], d['ms_per_step'], d['roofline']['kernel'], d['roofline']['frac'], d['cpu_baseline'].get('value'), d['cpu_baseline'].get('legs'))"
timeout -k 10 300 python bench.py --model cnn_deep --precision bf16 --steps 5 --warmup 2 --no-cpu-baseline --no-peaks \
    > $OUT/deep_bf16.json 2> $OUT/deep_bf16.err || { tail -5 $OUT/deep_bf16.err; exit 1; }
python3 -c "import json;d=json.load(open('$OUT/deep_bf16.json'));print('deep bf16', d['value'], d['ms_per_step'], d['roofline']['kernel'], d['roofline']['frac'], d['step_roofline'])"
echo r4-check-done
