#!/bin/bash
# Analysis aid: L2-miss (FETCH_SIZE) / write bytes and L2 hit rate of the Winograd forward of layer 2
# (40 x 200, 32 -> 32, BN + ReLU prologue) at B = 4096 under three unit orders: s = static XCD-contiguous,
# n = static blockIdx order (a library built with make AB=-DPCX_AB_WINO_SLOT=1), q = per-XCD work queue (WINO_QUEUE=1); one counter group
# per rocprofv3 pass.  SHAPE / MODES override.
set -o pipefail
cd "$(dirname "$0")"; mkdir -p ../gpurun_out
export TMPDIR=/tmp
OUT=$PWD/../gpurun_out/pmc_wino_l2; rm -rf $OUT; mkdir -p $OUT
SHAPE=${SHAPE:-"40 200 32 32 4096"}
for mode in ${MODES:-s n q}; do
  envs=""
  # (mode n: run against a library built with make AB=-DPCX_AB_WINO_SLOT=1)
  [ $mode = q ] && envs="WINO_QUEUE=1"
  i=0
  for grp in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum"; do
    i=$((i+1))
    env $envs timeout -s KILL 90 rocprofv3 --pmc $grp -f csv -d $OUT/m${mode}p$i -o run -- ./wino_bench $SHAPE 2 0 1 > $OUT/m${mode}p$i.log 2>&1 || { echo "pass $mode $i failed"; tail -5 $OUT/m${mode}p$i.log; exit 1; }
  done
  env $envs timeout -k 5 60 ./wino_bench $SHAPE 10 0 1 > $OUT/m${mode}time.log 2>&1 || { cat $OUT/m${mode}time.log; exit 1; }
  echo "mode $mode: $(tail -1 $OUT/m${mode}time.log)"
  python3 - $OUT $mode "$SHAPE" <<'PY'
import csv, glob, sys, collections
out, mode, shape = sys.argv[1:]
H, W, cin, cout, B = map(int, shape.split())
res = {}
for f in sorted(glob.glob("%s/m%sp*/**/*counter_collection.csv" % (out, mode), recursive=True)):
    acc = collections.OrderedDict()
    for r in csv.DictReader(open(f)):
        if "conv_wino_kernel" in r["Kernel_Name"]:
            acc.setdefault(r["Dispatch_Id"], collections.defaultdict(float))[r["Counter_Name"]] += float(r["Counter_Value"])
    if acc:
        res.update(list(acc.values())[-1])
xin, yout = B * cin * H * W * 4, B * cout * H * W * 4
f2, w = 2 * res.get("FETCH_SIZE", 0) * 1024, res.get("WRITE_SIZE", 0) * 1024
print("  ", " ".join("%s=%.4g" % kv for kv in sorted(res.items())),
      "| fetch x2 / input %.3f, write / output %.3f, (fetch x2 + write) / (input + output) %.3f" % (f2 / xin, w / yout, (f2 + w) / (xin + yout)))
PY
done
