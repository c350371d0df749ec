#!/bin/bash
# Round-6 evidence on the GPU box (repo root), in two calls (each within gpurun's time limit):
#   part a: all GPU tests (FULLSIZE margins to JSON), the default bench line (CPU baseline with the
#           B = 4096 leg), both cnn_deep lines, rocprofv3 kernel stats of the cnn_small step;
#   part b: PMC traffic per plan label (FETCH_SIZE / WRITE_SIZE passes mapped by ROCTx labels) for
#           cnn_small and both cnn_deep lines, MFMA-busy + MOPS pass at B = 4096 for cnn_small.
# Output under gpurun_out/ev6b/ (EVOUT).
set -o pipefail
OUT=gpurun_out/${EVOUT:-ev6b}
mkdir -p $OUT
export TMPDIR=/tmp
PART=${1:-a}
if [ "$PART" = a ]; then
  export PCX_FULLSIZE_JSON=$(pwd)/$OUT/fullsize_parity.json
  timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/gpu_tests.log 2>&1
  rc=$?; tail -2 $OUT/gpu_tests.log; grep -E "^FAILED|Error" $OUT/gpu_tests.log | head -5; [ $rc -eq 0 ] || exit 1
  timeout -k 10 500 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -5 $OUT/bench.err; exit 1; }
  python3 -c "import json;d=json.load(open('$OUT/bench.json'));print('small', d['value'], d['ms_per_step'], d['roofline']['kernel'], d['roofline']['frac'], d['cpu_baseline'].get('value'))"
  for prec in bf16 fp32; do
    timeout -k 10 300 python bench.py --model cnn_deep --precision $prec --steps 5 --warmup 2 --no-cpu-baseline --no-peaks \
        > $OUT/deep_$prec.json 2> $OUT/deep_$prec.err || { tail -5 $OUT/deep_$prec.err; exit 1; }
    python3 -c "import json;d=json.load(open('$OUT/deep_$prec.json'));print('deep $prec', d['value'], d['ms_per_step'], d['roofline']['kernel'], d['roofline']['frac'])"
  done
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $(pwd)/$OUT/trace -o run -- \
      python3 $(pwd)/bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-peaks --no-kernel-timing \
      > $OUT/bench_trace.json 2> $OUT/bench_trace.err || exit 1
  echo evidence-a-done
else
  bash scripts/pmc_deep.sh $OUT/pmc_small cnn_small/fp32 || exit 1
  bash scripts/pmc_deep.sh $OUT/pmc_deep_bf16 cnn_deep/bf16 --model cnn_deep --precision bf16 || exit 1
  bash scripts/pmc_deep.sh $OUT/pmc_deep_fp32 cnn_deep/fp32 --model cnn_deep --precision fp32 || exit 1
  bash scripts/pmc_busy4096.sh $OUT/busy_small cnn_small/fp32 || exit 1
  echo evidence-b-done
fi
