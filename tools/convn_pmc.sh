#!/bin/bash
# SQ stall counters of the channel-last conv kernels on one block-0 shape (analysis aid).
set -eo pipefail
export TMPDIR=/tmp
ROOT=$(pwd)
OUT=gpurun_out/convn_pmc
mkdir -p $OUT
for m in 0 1 2; do
  timeout -k 10 120 python3 tools/convn_bench.py --mode $m --shape ${SHAPE:-4096,64,64,20,100,3,1,1}
done
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY \
    SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT -f csv -d "$ROOT/$OUT/sq" -o run -- \
    python3 "$ROOT/tools/convn_bench.py" --mode 0 --iters 2 --shape ${SHAPE:-4096,64,64,20,100,3,1,1} > /dev/null 2> $OUT/sq.err
python3 - $OUT <<'PY'
import csv, glob, sys, collections
f = glob.glob(sys.argv[1] + "/sq/**/*counter_collection.csv", recursive=True)[0]
acc = collections.defaultdict(lambda: collections.defaultdict(float))
for r in csv.DictReader(open(f)):
    if "convn_kernel" in r["Kernel_Name"]:
        acc[r["Dispatch_Id"]][r["Counter_Name"]] += float(r["Counter_Value"])
for d, c in list(acc.items())[-1:]:
    for k, v in sorted(c.items()): print("%-28s %.4g" % (k, v))
PY
