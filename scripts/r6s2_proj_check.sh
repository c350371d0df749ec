#!/bin/bash
# Round 6 (session 2): model / trainer / DDP GPU tests, then rocprofv3 kernel stats of the cnn_small step
# (projection kernels printed; compared with the previous library's profiles/r6_final_kernel_stats.csv).
set -o pipefail
O=gpurun_out/${1:-pj}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_model_gpu.py tests/test_trainer_gpu.py tests/test_ddp_gpu.py \
    tests/test_fullsize_parity_gpu.py tests/test_small_shapes_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread \
    > $O/tests.log 2>&1
rc=$?; tail -1 $O/tests.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 240 rocprofv3 --kernel-trace --stats -f csv -d $PWD/$O/prof -o run -- \
    python3 $PWD/bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-peaks --no-kernel-timing \
    > $O/bench.json 2> $O/bench.err || exit 1
python3 - $O/prof <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + '/**/run_kernel_stats.csv', recursive=True)[0]
for r in csv.DictReader(open(f)):
    if 'proj' in r['Name'] or 'bn1d' in r['Name']:
        print(r['Name'][:60], r['Calls'], round(float(r['AverageNs']) / 1e3, 1), 'us')
PY
echo proj-done
