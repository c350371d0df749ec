#!/bin/bash
# cnn_small iteration check: Winograd weight-gradient cross-check (tools/run_ww.sh), the cnn_small
# model / engine GPU tests, then the headline bench line with its largest kernels.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 bash tools/run_ww.sh > gpurun_out/ww.txt 2>&1; rc=$?; cat gpurun_out/ww.txt | cut -c1-200
[ $rc -eq 0 ] || { echo "ww rc=$rc"; exit 1; }
timeout -k 10 400 python -u -m pytest tests/test_model_gpu.py tests/test_wino_engine_gpu.py tests/test_small_shapes_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/t_small.log 2>&1
rc=$?; tail -2 gpurun_out/t_small.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 300 python bench.py --no-cpu-baseline --no-peaks > gpurun_out/bench.json 2> gpurun_out/bench.err || { tail -5 gpurun_out/bench.err; exit 1; }
python3 - <<'PY'
import json
d=json.load(open("gpurun_out/bench.json")); print("cnn_small", d["value"], d["ms_per_step"], d["roofline"]["kernel"], d["roofline"]["frac"])
k=d["kernels"]; agg={n: v["avg_ms"]*v["launches"]/d["steps"] for n,v in k.items()}
print(sorted(((round(v,2),n) for n,v in agg.items()), reverse=True)[:16])
PY
