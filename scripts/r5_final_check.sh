#!/bin/bash
# HEAD check on the GPU box: every -m gpu test, smoke(), one default bench line (no CPU leg)
set -o pipefail
OUT=gpurun_out/final_check
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1
rc=$?; tail -2 $OUT/gpu_tests.log; grep -E "^FAILED|Error" $OUT/gpu_tests.log | head -5; [ $rc -eq 0 ] || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.log 2>&1 || { tail -5 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
timeout -k 10 300 python bench.py --no-cpu-baseline > $OUT/bench.json 2> $OUT/bench.err || { tail -5 $OUT/bench.err; exit 1; }
python3 -c "import json;d=json.load(open('$OUT/bench.json'));print('small', d['value'], d['ms_per_step'], d['roofline']['kernel'], d['roofline']['frac'])"
echo final-check-done
