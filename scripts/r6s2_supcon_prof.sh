#!/bin/bash
# Round 6 (session 2): rocprofv3 kernel stats of the cnn_small step with the in-tree library and a variant build
# (the SupCon kernels are launched by the loss module, outside the plan's labelled kernel table).
# Usage: scripts/r6s2_supcon_prof.sh OUTDIR variant_dir
set -o pipefail
O=gpurun_out/${1:-sc}; V=$2
mkdir -p $O
export TMPDIR=/tmp
for arm in base var base2 var2; do
  lib=""; case $arm in var*) lib=$PWD/$V/libpcx.so;; esac
  PCX_LIB_PATH=$lib timeout -k 10 240 rocprofv3 --kernel-trace --stats -f csv -d $PWD/$O/$arm -o run -- \
      python3 $PWD/bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-peaks --no-kernel-timing \
      > $O/$arm.json 2> $O/$arm.err || exit 1
  python3 - $O/$arm <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + '/**/run_kernel_stats.csv', recursive=True)[0]
for r in csv.DictReader(open(f)):
    if 'supcon' in r['Name'] or 'sum_splits' in r['Name']:
        print(sys.argv[1].split('/')[-1], r['Name'][:60], r['Calls'], round(float(r['AverageNs']) / 1e3, 1), 'us')
PY
done
echo prof-done
