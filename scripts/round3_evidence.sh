#!/bin/bash
# Round-3 evidence on the GPU box (repo root), in two calls (each within gpurun's time limit):
#   part a: all GPU tests, the default bench line (with the CPU baseline), both cnn_deep lines,
#           rocprofv3 kernel stats + FETCH/WRITE_SIZE + stall passes for cnn_small;
#   part b: PMC traffic per plan label for cnn_deep bf16 and fp32, kernel stats of the bf16 step.
# Output under gpurun_out/ev3/.
set -o pipefail
OUT=gpurun_out/ev3
mkdir -p $OUT
export TMPDIR=/tmp
PART=${1:-a}
if [ "$PART" = a ]; then
  timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/gpu_tests.log 2>&1
  rc=$?; tail -2 $OUT/gpu_tests.log; [ $rc -eq 0 ] || exit 1
  timeout -k 10 400 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -5 $OUT/bench.err; exit 1; }
  python3 -c "import json;d=json.load(open('$OUT/bench.json'));print('small', d['value'], d['ms_per_step'], d['roofline']['kernel'], d['roofline']['frac'])"
  for prec in fp32 bf16; do
    timeout -k 10 300 python bench.py --model cnn_deep --precision $prec --steps 5 --warmup 2 --no-cpu-baseline --no-peaks \
        > $OUT/deep_$prec.json 2> $OUT/deep_$prec.err || { tail -5 $OUT/deep_$prec.err; exit 1; }
    python3 -c "import json;d=json.load(open('$OUT/deep_$prec.json'));print('deep $prec', d['value'], d['ms_per_step'], d['roofline']['kernel'], d['roofline']['frac'])"
  done
  bash scripts/gpu_profile_all.sh $OUT/prof || exit 1
  echo evidence-a-done
else
  bash scripts/pmc_deep.sh $OUT/pmc_deep_bf16 cnn_deep/bf16 --model cnn_deep --precision bf16 || exit 1
  bash scripts/pmc_deep.sh $OUT/pmc_deep_fp32 cnn_deep/fp32 --model cnn_deep --precision fp32 || exit 1
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $(pwd)/$OUT/deep_trace -o run -- \
      python3 $(pwd)/bench.py --model cnn_deep --precision bf16 --steps 3 --warmup 1 --no-cpu-baseline --no-peaks --no-kernel-timing \
      > $OUT/deep_trace.json 2> $OUT/deep_trace.err || exit 1
  echo evidence-b-done
fi
