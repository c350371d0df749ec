#!/bin/bash
# Analysis aid: instruction mix and wait counters of one standalone kernel run (one rocprofv3 --pmc pass of 8 SQ
# counters + one of LDS counters).  Usage: tools/pmc_mix.sh NAME KERNEL_SUBSTRING -- command...
set -o pipefail
NAME=$1; KS=$2; shift 3
export TMPDIR=/tmp
OUT=gpurun_out/pmc_mix/$NAME; rm -rf $OUT; mkdir -p $OUT
i=0
for grp in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU" \
           "SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_VMEM SQ_ACTIVE_INST_ANY SQ_INST_LEVEL_LDS"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $grp -f csv -d $OUT/p$i -o run -- "$@" > $OUT/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $OUT/p$i.log; exit 1; }
done
python3 - $OUT "$KS" <<'PY'
import csv, glob, sys, collections
out, ks = sys.argv[1:]
res = {}
for f in sorted(glob.glob(out + "/p*/**/*counter_collection.csv", recursive=True)):
    acc = collections.OrderedDict()
    for r in csv.DictReader(open(f)):
        if ks in r["Kernel_Name"]:
            acc.setdefault(r["Dispatch_Id"], collections.defaultdict(float))[r["Counter_Name"]] += float(r["Counter_Value"])
    if acc:
        res.update(list(acc.values())[-1])
w = res.get("SQ_WAVE_CYCLES", 1)
m = res.get("SQ_INSTS_MFMA", 1)
print(" ".join(f"{k}={v:.4g}" for k, v in sorted(res.items())))
print(f"per MFMA: VALU {res.get('SQ_INSTS_VALU', 0) / m:.2f} LDS {res.get('SQ_INSTS_LDS', 0) / m:.2f} SALU {res.get('SQ_INSTS_SALU', 0) / m:.2f} "
      f"VMEM {res.get('SQ_INSTS_VMEM', 0) / m:.2f}; of wave cycles: WAIT_INST_ANY {res.get('SQ_WAIT_INST_ANY', 0) / w:.3f} "
      f"WAIT_ANY {res.get('SQ_WAIT_ANY', 0) / w:.3f} ACTIVE_VALU {res.get('SQ_ACTIVE_INST_VALU', 0) / w:.3f} "
      f"ACTIVE_LDS {res.get('SQ_ACTIVE_INST_LDS', 0) / w:.3f} WAIT_INST_LDS {res.get('SQ_WAIT_INST_LDS', 0) / w:.3f} "
      f"ACTIVE_ANY {res.get('SQ_ACTIVE_INST_ANY', 0) / w:.3f} bank_conflict/LDS {res.get('SQ_LDS_BANK_CONFLICT', 0) / max(res.get('SQ_INSTS_LDS', 1), 1):.3f}")
PY
