#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/pmcstem
mkdir -p $OUT
timeout -k 10 200 bash tools/run_stem.sh > $OUT/stem.txt 2>&1 || { cat $OUT/stem.txt; exit 1; }
grep -E "stem B|MISMATCH|backward:|stem path" $OUT/stem.txt
cd tools
timeout -s KILL 60 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU GRBM_GUI_ACTIVE -f csv -d ../$OUT/p1 -o run -- ./stem_bench 4096 40 200 1 > ../$OUT/p1.log 2>&1 || exit 1
timeout -s KILL 60 rocprofv3 --pmc TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum TCC_EA0_RDREQ_sum TCC_HIT_sum -f csv -d ../$OUT/p2 -o run -- ./stem_bench 4096 40 200 1 > ../$OUT/p2.log 2>&1 || exit 1
echo pmc-done
