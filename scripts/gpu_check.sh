#!/bin/bash
# GPU-box check of the current tree: the -m gpu suite, then (if it passed) one default bench line.
# Usage: bash scripts/gpu_check.sh [pytest selection...]   (output under gpurun_out/)
set -o pipefail
mkdir -p gpurun_out
SEL=${@:-tests}
timeout -k 10 1000 python -u -m pytest $SEL -m gpu -v --timeout 300 --timeout-method thread \
    > gpurun_out/gpu_tests.log 2>&1
rc=$?
tail -25 gpurun_out/gpu_tests.log
[ $rc -eq 0 ] || exit $rc
if [ -z "$NO_BENCH" ]; then
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-peaks > gpurun_out/bench.json 2> gpurun_out/bench.err || { tail -20 gpurun_out/bench.err; exit 1; }
  python3 -c "
import json;d=json.load(open('gpurun_out/bench.json'));print(d['value'], d['ms_per_step'], d['roofline']);print({k:v['avg_ms'] for k,v in d['kernels'].items()})"
fi
