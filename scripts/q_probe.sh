#!/bin/bash
# round-4 analysis: unit order of the Winograd convs (static vs per-XCD queue): PMC probe, standalone
# timing of every cnn_small Winograd shape both ways, the GPU tests, a same-box bench A/B
set -o pipefail
mkdir -p gpurun_out
( cd tools && MODES="s q" timeout -k 10 300 ./pmc_wino_l2.sh ) > gpurun_out/pmc_wino_l2.txt 2>&1 || { cat gpurun_out/pmc_wino_l2.txt; exit 1; }
cat gpurun_out/pmc_wino_l2.txt
for q in 0 1; do echo "WINO_QUEUE=$q"; ( cd tools && WINO_QUEUE=$q timeout -k 10 200 ./run_wino.sh ) || exit 1; done > gpurun_out/run_wino_q.txt 2>&1 || { cat gpurun_out/run_wino_q.txt; exit 1; }
cat gpurun_out/run_wino_q.txt
timeout -k 10 420 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/q_gpu_tests.txt 2>&1 || { tail -30 gpurun_out/q_gpu_tests.txt; exit 1; }
tail -2 gpurun_out/q_gpu_tests.txt
NK=16 ROUNDS=2 timeout -k 10 400 scripts/ab_bench.sh gpurun_out/ab_q PCX_NO_WINO_QUEUE=1:
