#!/bin/bash
# PMC passes over ww_bench (Winograd weight gradient) on one shape (analysis aid): counters only, one pass per group
set -o pipefail
cd "$(dirname "$0")"; mkdir -p ../gpurun_out
export LD_LIBRARY_PATH=$PWD/../phoneme_contrast_amd:$LD_LIBRARY_PATH TMPDIR=/tmp
OUT=$PWD/../gpurun_out/pmc_ww; mkdir -p $OUT
SHAPE=${SHAPE:-"40 200 32 32 4096 2 1"}
i=0
for grp in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE" \
           "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVES SQ_INSTS_BRANCH" \
           "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_FLAT SQ_INST_CYCLES_VMEM SQ_LDS_IDX_ACTIVE SQ_INST_LEVEL_LDS"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $grp -f csv -d $OUT/p$i -o run -- ./ww_bench $SHAPE > $OUT/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $OUT/p$i.log; exit 1; }
done
echo done
