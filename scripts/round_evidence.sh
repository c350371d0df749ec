#!/bin/bash
# Round-end evidence on the GPU box (repo root): GPU tests, the default bench line (with the CPU
# baseline), rocprofv3 kernel stats + FETCH/WRITE_SIZE passes + one stall-counter pass.
# Output under gpurun_out/ev/; copy the summaries into profiles/ afterwards.
set -eo pipefail
OUT=gpurun_out/ev
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/gpu_tests.log 2>&1
tail -2 $OUT/gpu_tests.log
timeout -k 10 400 python bench.py > $OUT/bench.json 2> $OUT/bench.err
cat $OUT/bench.json
bash scripts/gpu_profile_all.sh $OUT/prof
cp $OUT/prof/trace/run_kernel_stats.csv $OUT/kernel_stats.csv
echo evidence-done
