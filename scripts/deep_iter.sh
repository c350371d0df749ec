#!/bin/bash
# Iteration check for the cnn_deep bf16 path on the GPU box: stem cross-check, bf16 / deep / config-5
# GPU tests, the bf16 bench line with its largest kernels.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 bash tools/run_stem.sh > gpurun_out/stem.txt 2>&1; rc=$?
grep -E "stem B|MISMATCH|backward:|stem path|rel |after|failed" gpurun_out/stem.txt
[ $rc -eq 0 ] || { echo "stem check rc=$rc"; exit 1; }
timeout -k 10 400 python -u -m pytest tests/test_deep_bf16_gpu.py tests/test_config5_gpu.py tests/test_deep_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/t_deep.log 2>&1
rc=$?; tail -3 gpurun_out/t_deep.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 200 python bench.py --model cnn_deep --precision bf16 --steps 5 --warmup 2 --no-cpu-baseline --no-peaks > gpurun_out/deep_bf16.json 2> gpurun_out/deep_bf16.err || { tail -5 gpurun_out/deep_bf16.err; exit 1; }
python3 - <<'PY'
import json
d=json.load(open("gpurun_out/deep_bf16.json")); print("bf16", d["value"], d["ms_per_step"])
k=d["kernels"]; agg={n: v["avg_ms"]*v["launches"]/d["steps"] for n,v in k.items()}
print(sorted(((round(v,2),n) for n,v in agg.items()), reverse=True)[:30])
PY
