#!/bin/bash
# PMC passes (one counter group per run, counters only) over the channel-last conv micro-benchmark;
# prints the counters of the last convn_kernel dispatch of each pass.  Analysis aid.
export TMPDIR=/tmp
ROOT=$(pwd)
OUT=gpurun_out/convn_pmc
SHAPE=${SHAPE:-2048,256,256,20,100,3,1,1}
MODE=${MODE:-0}
rm -rf $OUT; mkdir -p $OUT
pass() {
  local name=$1; shift
  timeout -s KILL 60 rocprofv3 --pmc "$@" -f csv -d "$ROOT/$OUT/$name" -o run -- \
      python3 "$ROOT/tools/convn_bench.py" --mode $MODE --iters 2 --shape $SHAPE > /dev/null 2> $OUT/$name.err
  echo "pass $name rc=$?"
}
pass sq SQ_INSTS_VMEM_RD SQ_INST_LEVEL_VMEM SQ_INSTS_LDS SQ_INST_LEVEL_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_ANY
pass tcp TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum
pass tcc TCC_HIT_sum TCC_MISS_sum
pass ta TA_ADDR_STALLED_BY_TC_CYCLES_sum TA_DATA_STALLED_BY_TC_CYCLES_sum
python3 - $OUT <<'PY'
import csv, glob, sys, collections
for f in sorted(glob.glob(sys.argv[1] + "/*/**/*counter_collection.csv", recursive=True)):
    acc = collections.OrderedDict()
    for r in csv.DictReader(open(f)):
        if "convn_kernel" in r["Kernel_Name"]:
            acc.setdefault(r["Dispatch_Id"], collections.defaultdict(float))[r["Counter_Name"]] += float(r["Counter_Value"])
    if acc:
        d = list(acc.values())[-1]
        print(" ".join("%s=%.4g" % kv for kv in sorted(d.items())))
PY
