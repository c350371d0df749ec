#!/bin/bash
# Same-box A/B timing of library variants (run on the GPU box from the repo root): the cnn_small bench
# line for the in-tree library and each variant build (a directory holding a libpcx.so, e.g. from
# tools/wb_ko.sh), alternating ROUNDS times so box drift hits every variant alike.
#   scripts/ab_bench.sh <out dir> <variant dir>...      (env "VAR=value" prefixes allowed as <k>=<v>:dir)
set -o pipefail
OUT=$1; shift
mkdir -p "$OUT"
for r in $(seq 1 ${ROUNDS:-2}); do
  for v in base "$@"; do
    tag=$(echo "$v" | tr '/=:' '___')
    if [ "$v" = base ]; then envs=""; else
      envs=""; dir="$v"
      if [[ "$v" == *:* ]]; then envs="${v%%:*}"; dir="${v#*:}"; fi
      [ -n "$dir" ] && envs="$envs PCX_LIB_PATH=$PWD/$dir/libpcx.so"
    fi
    env $envs timeout -k 10 300 python bench.py --no-cpu-baseline --no-peaks ${BENCH_ARGS:-} > "$OUT/$tag.$r.json" 2> "$OUT/$tag.$r.err" || { tail -3 "$OUT/$tag.$r.err"; exit 1; }
    python3 -c "import json,sys;d=json.load(open('$OUT/$tag.$r.json'));k=d['kernels'];print('$tag', $r, d['value'], d['ms_per_step'], ' '.join(f'{n}={k[n][\"avg_ms\"]}' for n in list(k)[:${NK:-6}]))"
  done
done
echo ab-done
