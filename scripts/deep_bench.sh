#!/bin/bash
# cnn_deep fp32 and bf16 bench lines (B = 4096) with per-kernel timing, on the GPU box.
set -o pipefail
mkdir -p gpurun_out
for prec in fp32 bf16; do
  timeout -k 10 300 python bench.py --model cnn_deep --precision $prec --steps 5 --warmup 2 --no-cpu-baseline --no-peaks \
      > gpurun_out/deep_$prec.json 2> gpurun_out/deep_$prec.err || { tail -20 gpurun_out/deep_$prec.err; exit 1; }
  python3 -c "
import json;d=json.load(open('gpurun_out/deep_$prec.json'));print('$prec', d['value'], d['ms_per_step'])
k=d['kernels']; agg={n: v['avg_ms']*v['launches']/d['steps'] for n,v in k.items()}
print(sorted(((round(v,2),n) for n,v in agg.items()), reverse=True)[:25])"
done
