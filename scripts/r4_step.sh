#!/bin/bash
# Round-4 GPU iteration (repo root): fused layer-2 backward cross-check, GPU tests, bench, MFMA-busy
# PMC passes.  Output under gpurun_out/$1.  Stops at the first failing step.
set -o pipefail
OUT=gpurun_out/${1:-r4}
mkdir -p $OUT
export TMPDIR=/tmp
export PCX_FULLSIZE_JSON=$(pwd)/$OUT/fullsize_parity.json
for c in "40 200 48 1" "20 100 24 1" "21 56 16 1" "40 200 4096 5"; do
  timeout -k 10 120 ./tools/wb_bench $c >> $OUT/wb.log 2>&1 || { echo "wb_bench $c failed rc=$?"; cat $OUT/wb.log; exit 1; }
done
cat $OUT/wb.log
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1
rc=$?; tail -3 $OUT/gpu_tests.log; grep -E "^FAILED|Error" $OUT/gpu_tests.log | head -5; [ $rc -eq 0 ] || exit 1
timeout -k 10 500 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -5 $OUT/bench.err; exit 1; }
python3 -c "import json;d=json.load(open('$OUT/bench.json'));print('small', d['value'], d['ms_per_step'], d['roofline']['kernel'], d['roofline']['frac'], d['cpu_baseline'].get('value'), [ (l['B'], l['samples_per_s']) for l in d['cpu_baseline'].get('legs', [])]); print({k: v['avg_ms'] for k, v in list(d['kernels'].items())[:12]})"
if [ "${2:-}" = pmc ]; then
  bash scripts/pmc_busy.sh $OUT/busy_small cnn_small/fp32 --batch 512 || exit 1
  bash scripts/pmc_busy.sh $OUT/busy_deep cnn_deep/fp32 --batch 512 --model cnn_deep --precision fp32 || exit 1
  cp gpurun_out/mfma_busy.json $OUT/
fi
echo r4-step-done
