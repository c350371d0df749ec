set -o pipefail
mkdir -p gpurun_out/y16dbg
for v in 1 0; do PCX_NO_Y16=$v timeout -k 10 300 python -u -m pytest -s -x -q "tests/test_deep_bf16_gpu.py::test_deep_bf16_step" -m gpu --timeout 200 --timeout-method thread > gpurun_out/y16dbg/t$v.log 2>&1; grep "bf16 residual" gpurun_out/y16dbg/t$v.log | sed "s/^/NOY16=$v /"; done
echo done
