#!/bin/bash
# Round-6 iteration on the GPU box: optional analysis tool, a subset of -m gpu tests, one bench line.
# Usage: scripts/r6_quick.sh TAG "pytest selection" [tool command]
set -o pipefail
OUT=gpurun_out/${1:-r6q}
mkdir -p $OUT
export TMPDIR=/tmp
if [ -n "$3" ]; then timeout -k 10 240 $3 > $OUT/tool.txt 2>&1 || { tail -5 $OUT/tool.txt; exit 1; }; tail -30 $OUT/tool.txt; fi
if [ -n "$2" ]; then
  timeout -k 10 600 python -u -m pytest $2 -m gpu -x -q -s --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1
  rc=$?; grep -E "passed|failed" $OUT/gpu_tests.log | tail -2; grep -E "^FAILED|Error" $OUT/gpu_tests.log | head -5; [ $rc -eq 0 ] || exit 1
fi
timeout -k 10 300 python bench.py --no-cpu-baseline ${BENCH_ARGS} > $OUT/bench.json 2> $OUT/bench.err || { tail -5 $OUT/bench.err; exit 1; }
python3 - $OUT/bench.json <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
print("value", d["value"], "ms", d["ms_per_step"], "roof", d["roofline"]["kernel"], d["roofline"]["frac"], d["measured_peaks"])
for k, v in list(d["kernels"].items())[:24]:
    print(f"  {k:18s} {v['avg_ms']:.4f} ms  exec {v.get('exec_frac', '')}  gbps {v.get('alg_gbps', '')}")
PY
echo quick-done
