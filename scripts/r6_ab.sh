#!/bin/bash
# Same-box A/B: the default bench line with the in-tree library, then with tools/ab/libpcx.so (an analysis
# build, make AB=... LIB=tools/ab/libpcx.so BUILD=tools/ab/obj).  Usage: scripts/r6_ab.sh TAG [pytest selection]
set -o pipefail
OUT=gpurun_out/${1:-r6ab}
mkdir -p $OUT
export TMPDIR=/tmp
if [ -n "$2" ]; then
  timeout -k 10 600 python -u -m pytest $2 -m gpu -x -q -s --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1
  rc=$?; grep -E "passed|failed" $OUT/gpu_tests.log | tail -2; grep -E "^FAILED|Error" $OUT/gpu_tests.log | head -5; [ $rc -eq 0 ] || exit 1
fi
for arm in A B A2 B2; do
  lib=""; case $arm in B*) lib=$PWD/tools/ab/libpcx.so;; esac
  PCX_LIB_PATH=$lib timeout -k 10 300 python bench.py --no-cpu-baseline --no-peaks ${BENCH_ARGS} > $OUT/bench_$arm.json 2> $OUT/bench_$arm.err || { tail -5 $OUT/bench_$arm.err; exit 1; }
done
python3 - $OUT <<'PY'
import json, sys
d = {a: json.load(open(f"{sys.argv[1]}/bench_{a}.json")) for a in ("A", "B", "A2", "B2")}
print(" ".join(f"{a}: {v['value']} ({v['ms_per_step']} ms)" for a, v in d.items()))
for k in list(d["A"]["kernels"])[:26]:
    print(f"  {k:18s} " + "  ".join(f"{d[a]['kernels'].get(k, {}).get('avg_ms', 0):.4f}" for a in d))
PY
echo ab-done
