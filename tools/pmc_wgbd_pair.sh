#!/bin/bash
# Analysis aid: L2-miss / write bytes of the fused layer-2 backward (wgbd_wino, pooled dz, B = 4096)
# with the XCD-paired strips and without (a library built with make AB=-DPCX_AB_WGBD_UNPAIRED=1), plus standalone timing; one counter per pass
set -o pipefail
cd "$(dirname "$0")"; mkdir -p ../gpurun_out
export TMPDIR=/tmp
OUT=$PWD/../gpurun_out/pmc_wgbd_pair; rm -rf $OUT; mkdir -p $OUT
for mode in p u; do
  envs=""  # (mode u: run against a library built with make AB=-DPCX_AB_WGBD_UNPAIRED=1)
  for c in FETCH_SIZE WRITE_SIZE; do
    env $envs timeout -s KILL 90 rocprofv3 --pmc $c -f csv -d $OUT/$mode$c -o run -- ./wb_bench 40 200 4096 2 1 > $OUT/$mode$c.log 2>&1 || { echo "pass $mode $c failed"; tail -5 $OUT/$mode$c.log; exit 1; }
  done
  env $envs timeout -k 5 60 ./wb_bench 40 200 4096 10 1 > $OUT/${mode}time.log 2>&1 || { cat $OUT/${mode}time.log; exit 1; }
  echo "mode $mode: $(tail -1 $OUT/${mode}time.log)"
  python3 - $OUT $mode <<'PY'
import csv, glob, sys, collections
out, mode = sys.argv[1:]
res = {}
for f in sorted(glob.glob("%s/%s*/**/*counter_collection.csv" % (out, mode), recursive=True)):
    acc = collections.OrderedDict()
    for r in csv.DictReader(open(f)):
        if "wgbd_wino_kernel" in r["Kernel_Name"]:
            acc.setdefault(r["Dispatch_Id"], collections.defaultdict(float))[r["Counter_Name"]] += float(r["Counter_Value"])
    if acc:
        res.update(list(acc.values())[-1])
f2, w = 2 * res.get("FETCH_SIZE", 0) * 1024, res.get("WRITE_SIZE", 0) * 1024
print("   fetch x2 %.2f GB, write %.2f GB, total %.2f GB" % (f2 / 1e9, w / 1e9, (f2 + w) / 1e9))
PY
done
