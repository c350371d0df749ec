# GPU-box check: deep parity tests (fp32 + bf16 + conv2d engine) and one cnn_deep bench per precision
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_conv2d_gpu.py tests/test_deep_gpu.py tests/test_deep_bf16_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/t.log 2>&1; tail -2 gpurun_out/t.log
for pr in fp32 bf16; do
timeout -k 10 300 python bench.py --model cnn_deep --precision $pr --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/bench_deep_$pr.json 2> gpurun_out/bench_deep_$pr.err
python3 -c "
import json;d=json.load(open('gpurun_out/bench_deep_$pr.json'));print('$pr', d['value'],d['ms_per_step'])
agg={}
for k,v in d['kernels'].items():
    b=k.rstrip('0123456789').rstrip('_L'); agg[b]=agg.get(b,0)+v['avg_ms']*v['launches']/d['steps']
print({k:round(v,2) for k,v in sorted(agg.items(), key=lambda kv:-kv[1])})"
done
