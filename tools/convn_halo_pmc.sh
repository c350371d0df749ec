#!/bin/bash
# PMC passes over the channel-last conv micro-benchmark (halo kernel at the block-0 shape, or the per-tap
# kernel in a library built with make AB=-DPCX_AB_NO_CONVN_HALO=1); one counter group per run.  Analysis aid: gpurun_out/convn_halo_pmc/
export TMPDIR=/tmp
ROOT=$(pwd)
OUT=gpurun_out/convn_halo_pmc${TAG:-}
SHAPE=${SHAPE:-4096,64,64,20,100,3,1,1}
MODE=${MODE:-0}
rm -rf $OUT; mkdir -p $OUT
timeout -k 5 120 python3 tools/convn_bench.py --mode $MODE --iters 10 --shape $SHAPE | tee $OUT/time.txt || exit 1
pass() {
  local name=$1; shift
  timeout -s KILL 90 rocprofv3 --pmc "$@" -f csv -d "$ROOT/$OUT/$name" -o run -- \
      python3 "$ROOT/tools/convn_bench.py" --mode $MODE --iters 2 --shape $SHAPE > /dev/null 2> $OUT/$name.err
  echo "pass $name rc=$?"
}
pass a SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_SALU
pass b SQ_WAVE_CYCLES SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INST_LEVEL_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_LDS_IDX_ACTIVE
pass c TA_ADDR_STALLED_BY_TC_CYCLES_sum TA_DATA_STALLED_BY_TC_CYCLES_sum TCC_HIT_sum TCC_MISS_sum
python3 - $OUT <<'PY'
import csv, glob, sys, collections
for f in sorted(glob.glob(sys.argv[1] + "/*/**/*counter_collection.csv", recursive=True)):
    acc = collections.OrderedDict()
    for r in csv.DictReader(open(f)):
        if "convn" in r["Kernel_Name"] and "pack" not in r["Kernel_Name"]:
            acc.setdefault(r["Dispatch_Id"], collections.defaultdict(float))[r["Counter_Name"]] += float(r["Counter_Value"])
    if acc:
        d = list(acc.values())[-1]
        w = d.get("SQ_WAVE_CYCLES", 0)
        print(" ".join("%s=%.4g" % (k, v / w if (w and k.startswith(("SQ_WAIT", "SQ_ACTIVE", "SQ_BUSY"))) else v) for k, v in sorted(d.items())))
PY
