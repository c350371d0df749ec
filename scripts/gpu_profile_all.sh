#!/bin/bash
# Full rocprofv3 evidence pass for the bench workload (run on the GPU box from the repo root):
# kernel trace + stats, FETCH_SIZE / WRITE_SIZE passes, one stall-counter pass; summaries under $OUT.
set -eo pipefail
OUT=${1:-gpurun_out/prof}
bash scripts/profile_gpu.sh "$OUT"
bash scripts/pmc_stalls.sh "$OUT"
python3 scripts/pmc_summary.py --stalls "$OUT/pmc_stall/run_counter_collection.csv" "$OUT/pmc_stalls.json" > /dev/null
