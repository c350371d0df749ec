#!/bin/bash
# PMC passes over wino_bench on one shape (analysis aid): counters only, one pass per group;
# prints the counters of the last Winograd dispatch of each pass
set -o pipefail
cd "$(dirname "$0")"; mkdir -p ../gpurun_out
export TMPDIR=/tmp
OUT=$PWD/../gpurun_out/pmc_wino; rm -rf $OUT; mkdir -p $OUT
SHAPE=${SHAPE:-"40 200 32 32 4096 2 0 1"}
i=0
for grp in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE" \
           "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVES SQ_INSTS_BRANCH" \
           "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_FLAT SQ_INST_CYCLES_VMEM SQ_LDS_IDX_ACTIVE SQ_INST_LEVEL_LDS" \
           "TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum TCC_HIT_sum TCC_MISS_sum" \
           "TA_BUSY_avr TA_ADDR_STALLED_BY_TC_CYCLES_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum SQ_WAIT_INST_LDS SQ_INSTS_SMEM SQ_INST_LEVEL_VMEM SQ_INSTS_VMEM"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $grp -f csv -d $OUT/p$i -o run -- ./wino_bench $SHAPE > $OUT/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $OUT/p$i.log; exit 1; }
done
python3 - $OUT <<'PY'
import csv, glob, sys, collections
for f in sorted(glob.glob(sys.argv[1] + "/*/**/*counter_collection.csv", recursive=True)):
    acc = collections.OrderedDict()
    for r in csv.DictReader(open(f)):
        if "conv_wino_kernel" in r["Kernel_Name"]:
            acc.setdefault(r["Dispatch_Id"], collections.defaultdict(float))[r["Counter_Name"]] += float(r["Counter_Value"])
    if acc:
        d = list(acc.values())[-1]
        print(" ".join("%s=%.4g" % kv for kv in sorted(d.items())))
PY
