#!/bin/bash
# Round 6 (session 2): every -m gpu test, smoke(), one default bench line, then optional analysis commands.
set -o pipefail
OUT=gpurun_out/${1:-r6s2full}; shift
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q -s --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1
rc=$?; grep -E "passed|failed" $OUT/gpu_tests.log | tail -2; grep -E "^FAILED|Error" $OUT/gpu_tests.log | head -5; [ $rc -eq 0 ] || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.log 2>&1 || { tail -5 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
timeout -k 10 300 python bench.py --no-cpu-baseline > $OUT/bench.json 2> $OUT/bench.err || { tail -5 $OUT/bench.err; exit 1; }
python3 -c "import json;d=json.load(open('$OUT/bench.json'));print('small', d['value'], d['ms_per_step'], d['roofline']['kernel'], d['roofline']['frac'])"
for c in "$@"; do echo "== $c"; timeout -k 10 120 bash -c "$c" || exit 1; done
echo full-done
