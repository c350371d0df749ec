#!/bin/bash
# round-4: XCD-paired strips in wgbd_wino -- engine tests, PMC / timing probe, same-box bench A/B
set -o pipefail
OUT=gpurun_out/pair; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_wino_engine_gpu.py -x -q --timeout 120 --timeout-method thread -k "fused" > $OUT/wb_tests.log 2>&1 || { tail -30 $OUT/wb_tests.log; exit 1; }
tail -1 $OUT/wb_tests.log
timeout -k 10 300 tools/pmc_wgbd_pair.sh || exit 1
NK=6 ROUNDS=2 timeout -k 10 400 scripts/ab_bench.sh $OUT/ab PCX_WGBD_UNPAIRED=1:
