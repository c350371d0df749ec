for e in 0 1 2 3 4 5; do
  PCX_WGRAD_EXPT=$e timeout -k 10 120 python bench.py --no-cpu-baseline --steps 5 > gpurun_out/e$e.json 2>/dev/null
  python3 -c "
import json;d=json.load(open('gpurun_out/e$e.json'));print('expt $e', {k:v['avg_ms'] for k,v in d['kernels'].items() if k.startswith('wgrad_L') and k!='wgrad_L1'})"
done
