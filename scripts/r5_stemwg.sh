#!/bin/bash
# stem weight-gradient slice count A/B (PCX_STEM_WG_SLICES: target slices; default 1024 MFMA form, 256 fp32)
set -o pipefail
OUT=gpurun_out/${1:-r5stemwg}
mkdir -p $OUT
export TMPDIR=/tmp
for prec in bf16 fp32; do
for v in 0 768 2048 4096 0; do
  PCX_STEM_WG_SLICES=$v timeout -k 10 300 python bench.py --model cnn_deep --precision $prec --steps 4 --warmup 2 --no-cpu-baseline --no-peaks \
      > $OUT/deep_${prec}_$v.json 2> $OUT/deep_${prec}_$v.err || { tail -5 $OUT/deep_${prec}_$v.err; exit 1; }
  python3 - $OUT/deep_${prec}_$v.json $v $prec <<'PY'
import json, sys
d = json.load(open(sys.argv[1])); k = d['kernels']
print('stemwg', sys.argv[3], sys.argv[2], d['value'], d['ms_per_step'], {n: round(v['avg_ms'], 3) for n, v in k.items() if n in ('wgrad_L0',)})
PY
done
done
echo done
