mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_model_gpu.py tests/test_deep_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/t.log 2>&1; tail -3 gpurun_out/t.log
for cfg in ${CFGS:-default}; do
  if [ $cfg = default ]; then unset PCX_WG32; else export PCX_WG32=$cfg; fi
  timeout -k 10 120 python bench.py --no-cpu-baseline --steps 5 > gpurun_out/w.json 2>gpurun_out/w.err || { tail -5 gpurun_out/w.err; exit 1; }
  python3 -c "
import json;d=json.load(open('gpurun_out/w.json'));print('$cfg', d['value'], {k:v['avg_ms'] for k,v in d['kernels'].items() if k.startswith('wgrad')})"
done
