#!/bin/bash
# cnn_deep iteration check (both precisions): deep model tests incl. the full-size fp32 parity test,
# then both bench lines with their largest kernels.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_deep_bf16_gpu.py tests/test_config5_gpu.py tests/test_deep_gpu.py tests/test_conv2d_gpu.py "tests/test_fullsize_parity_gpu.py::test_cnn_deep_fp32_b4096_matches_float64" -x -q --timeout 120 --timeout-method thread > gpurun_out/t_deep2.log 2>&1
rc=$?; tail -3 gpurun_out/t_deep2.log; [ $rc -eq 0 ] || exit 1
for prec in fp32 bf16; do
  timeout -k 10 300 python bench.py --model cnn_deep --precision $prec --steps 5 --warmup 2 --no-cpu-baseline --no-peaks > gpurun_out/deep_$prec.json 2> gpurun_out/deep_$prec.err || { tail -5 gpurun_out/deep_$prec.err; exit 1; }
  python3 - $prec <<'PY'
import json, sys
p = sys.argv[1]
d=json.load(open(f"gpurun_out/deep_{p}.json")); print(p, d["value"], d["ms_per_step"])
k=d["kernels"]; agg={n: v["avg_ms"]*v["launches"]/d["steps"] for n,v in k.items()}
print(sorted(((round(v,2),n) for n,v in agg.items()), reverse=True)[:24])
PY
done
