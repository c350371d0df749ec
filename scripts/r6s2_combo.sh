set -o pipefail
bash scripts/r6s2_ab.sh s2ab8 "tests/test_wino_engine_gpu.py tests/test_model_gpu.py tests/test_fullsize_parity_gpu.py tests/test_deep_gpu.py tests/test_deep_bf16_gpu.py tests/test_conv2d_gpu.py tests/test_small_shapes_gpu.py" tools/ab6 tools/ab7 || exit 1
BENCH_ARGS="--model cnn_deep --precision fp32 --steps 3 --warmup 1" ROUNDS=1 NK=12 bash scripts/ab_bench.sh gpurun_out/s2ab8/fp32 tools/ab7 || exit 1
BENCH_ARGS="--model cnn_deep --precision bf16 --steps 5 --warmup 2" ROUNDS=1 NK=12 bash scripts/ab_bench.sh gpurun_out/s2ab8/bf16 tools/ab7 || exit 1
