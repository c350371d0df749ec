#!/bin/bash
# rocprofv3 kernel trace of the cnn_deep bench (precision $1, default bf16) -> gpurun_out/deep_trace_<prec>/
# and a per-kernel summary (calls, total ms per step, average us) on stdout.
set -eo pipefail
export TMPDIR=/tmp
PREC=${1:-bf16}
ROOT=$(pwd)
OUT=gpurun_out/deep_trace_$PREC
mkdir -p "$OUT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d "$ROOT/$OUT" -o run -- \
    python3 "$ROOT/bench.py" --model cnn_deep --precision "$PREC" --steps 3 --warmup 1 --no-cpu-baseline \
    --no-kernel-timing --no-peaks > "$ROOT/$OUT/bench.json" 2> "$ROOT/$OUT/bench.err"
python3 - "$OUT" <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True)[0]
rows = list(csv.DictReader(open(f)))
rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
for r in rows[:40]:
    print("%8.3f ms/step %6d calls %9.1f us  %s" % (float(r["TotalDurationNs"]) / 4e6, int(r["Calls"]),
          float(r["AverageNs"]) / 1e3, r["Name"][:150]))
PY
