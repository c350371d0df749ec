# GPU-box check: the full -m gpu suite and one default cnn_small bench line with per-kernel times
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/t.log 2>&1; tail -2 gpurun_out/t.log
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench.json 2> gpurun_out/bench.err
python3 -c "
import json;d=json.load(open('gpurun_out/bench.json'));print(d['value'],d['ms_per_step'],d['step_roofline']['mfma_fraction'],d['roofline']['kernel'],d['roofline']['frac'])
agg={}
for k,v in d['kernels'].items():
    b=k.rstrip('0123456789').rstrip('_L'); agg[b]=agg.get(b,0)+v['avg_ms']*v['launches']/d['steps']
print({k:round(v,2) for k,v in sorted(agg.items(), key=lambda kv:-kv[1])})"
