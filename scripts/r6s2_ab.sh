#!/bin/bash
# Round 6 (session 2): parity subset, then same-box timing of the in-tree library against variant builds.
# Usage: scripts/r6s2_ab.sh TAG "pytest selection" variant_dir...
set -o pipefail
OUT=gpurun_out/${1:-r6s2}; SEL=$2; shift 2
mkdir -p $OUT
export TMPDIR=/tmp
if [ -n "$SEL" ]; then
  timeout -k 10 700 python -u -m pytest $SEL -m gpu -x -q -s --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1
  rc=$?; grep -E "passed|failed" $OUT/gpu_tests.log | tail -2; grep -E "^FAILED|Error" $OUT/gpu_tests.log | head -5; [ $rc -eq 0 ] || exit 1
fi
ROUNDS=${ROUNDS:-2} NK=${NK:-10} bash scripts/ab_bench.sh $OUT "$@"
