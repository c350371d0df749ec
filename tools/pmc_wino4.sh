#!/bin/bash
# PMC passes of the F(4x3) conv vs F(2x2) in wino4_bench (analysis aid; GPU box, repo root)
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/pmc_w4
mkdir -p $OUT
S=${SHAPE:-"40 200 32 32 4096 2 0 1"}
i=0
for c in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_SALU GRBM_GUI_ACTIVE" \
         "SQ_WAVE_CYCLES SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_SCA SQ_INSTS_SMEM GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $c -f csv -d $(pwd)/$OUT/p$i -o run -- $(pwd)/tools/wino4_bench $S > $OUT/p$i.log 2>&1 || { echo "pass $i failed"; tail -3 $OUT/p$i.log; exit 1; }
done
python3 - <<'PY'
import csv, glob, collections
for i in (1, 2):
    f = glob.glob(f"gpurun_out/pmc_w4/p{i}/run_counter_collection.csv")[0]
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0].split("<")[0].split("::")[-1]
        agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
    for k, d in agg.items():
        if "conv_wino" not in k: continue
        w = d.get("SQ_WAVE_CYCLES", 1)
        print(i, k, {c: (round(v / w, 4) if c.startswith(("SQ_WAIT", "SQ_ACTIVE")) else v) for c, v in sorted(d.items())})
PY
