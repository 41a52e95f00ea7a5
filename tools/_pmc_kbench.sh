#!/bin/bash
# PMC passes (one rocprofv3 run per counter set) over tools/kbench.py --only $1; output gpurun_out/pmc_$1
set -o pipefail
export TMPDIR=/tmp
ROOT=$GRAFT_REPO_ROOT
ONLY=$1
OUT=$ROOT/gpurun_out/pmc_$ONLY
mkdir -p $OUT
cd /tmp
i=0
for set in "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVES GRBM_GUI_ACTIVE" \
           "SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE" \
           "SQ_INSTS_VALU_TRANS_F32 SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $set --kernel-trace -d $OUT/p$i -o c --output-format csv -- python3 $ROOT/tools/kbench.py --only $ONLY --iters 3 > $OUT/p$i.log 2>&1 || { echo "pass $i failed"; tail -3 $OUT/p$i.log; exit 1; }
done
cd $ROOT && python3 tools/pmc_summary.py $OUT --match "${2:-}"
