#!/bin/bash
# Round-6 check on the GPU box: every -m gpu test (margins printed), smoke(), one default bench line (no CPU
# leg).  Usage: scripts/r6_check.sh TAG [pytest selection]
set -o pipefail
OUT=gpurun_out/${1:-r6check}
SEL=${2:-tests}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest $SEL -m gpu -x -v -s --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1
rc=$?; grep -E "passed|failed" $OUT/gpu_tests.log | tail -2; grep -E "^FAILED|Error" $OUT/gpu_tests.log | head -5; [ $rc -eq 0 ] || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.log 2>&1 || { tail -5 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
timeout -k 10 300 python bench.py --no-cpu-baseline > $OUT/bench.json 2> $OUT/bench.err || { tail -5 $OUT/bench.err; exit 1; }
python3 -c "import json;d=json.load(open('$OUT/bench.json'));print('small', d['value'], d['ms_per_step'], d['roofline']['kernel'], d['roofline']['frac'], d['measured_peaks'])"
echo check-done
