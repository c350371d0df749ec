#!/bin/bash
# Round-5 iteration on the GPU box (repo root): all GPU tests (full-size margins to JSON), the bench line
# (B = 24 CPU leg only unless FULLCPU=1), cnn_deep lines on request (DEEP="bf16 fp32").  Output under
# gpurun_out/$1.  Stops at the first failing step.
set -o pipefail
OUT=gpurun_out/${1:-r5it}
mkdir -p $OUT
export TMPDIR=/tmp
export PCX_FULLSIZE_JSON=$(pwd)/$OUT/fullsize_parity.json
if [ -z "$NOTEST" ]; then
  timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1
  rc=$?; tail -2 $OUT/gpu_tests.log; grep -E "^FAILED|Error" $OUT/gpu_tests.log | head -5; [ $rc -eq 0 ] || exit 1
fi
CPU="--cpu-quick"; [ -n "$FULLCPU" ] && CPU=""
timeout -k 10 500 python bench.py $CPU > $OUT/bench.json 2> $OUT/bench.err || { tail -5 $OUT/bench.err; exit 1; }
python3 - "$OUT/bench.json" <<'PY'
import json, sys
d = json.load(open(sys.argv[1])); r = d["roofline"]
print("small", d["value"], d["ms_per_step"], r["kernel"], r["frac"], r.get("alg_equiv_frac"), d["step_roofline"]["mfma_fraction"])
k = d["kernels"]; agg = {n: v["avg_ms"] * v["launches"] / 5 for n, v in k.items()}
print(sorted(((round(v, 2), n, k[n].get("exec_frac")) for n, v in agg.items()), reverse=True)[:18])
PY
for m in ${DEEP:-}; do
  timeout -k 10 300 python bench.py --model cnn_deep --precision $m --steps 5 --warmup 2 --no-cpu-baseline --no-peaks \
      > $OUT/deep_$m.json 2> $OUT/deep_$m.err || { tail -5 $OUT/deep_$m.err; exit 1; }
  python3 -c "import json;d=json.load(open('$OUT/deep_$m.json'));r=d['roofline'];print('deep $m', d['value'], d['ms_per_step'], r['kernel'], r['frac'], d['step_roofline']['mfma_fraction'])"
done
echo r5-iter-done
