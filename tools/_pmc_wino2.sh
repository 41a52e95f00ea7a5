#!/bin/bash
# PMC passes over one wino2 shape (SHAPE env, default the VAE's 512² x 128 layer)
set -o pipefail
export TMPDIR=/tmp
ROOT=$GRAFT_REPO_ROOT
OUT=$ROOT/gpurun_out/pmc_wino2
mkdir -p $OUT
SH=${SHAPE:-8,128,128,512}
cd /tmp
timeout -s KILL 90 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_ANY SQ_WAVE_CYCLES GRBM_GUI_ACTIVE --kernel-trace -d $OUT/p1 -o c --output-format csv -- python3 $ROOT/tools/wino_time.py --shapes "$SH" --iters 2 > $OUT/p1.log 2>&1 || { echo "pass1 failed"; tail -3 $OUT/p1.log; exit 1; }
timeout -s KILL 90 rocprofv3 --pmc SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_LDS SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_ACTIVE_INST_ANY SQ_INSTS_VALU GRBM_GUI_ACTIVE --kernel-trace -d $OUT/p2 -o c --output-format csv -- python3 $ROOT/tools/wino_time.py --shapes "$SH" --iters 2 > $OUT/p2.log 2>&1 || { echo "pass2 failed"; tail -3 $OUT/p2.log; exit 1; }
cd $ROOT && python3 tools/pmc_summary.py $OUT --match wino2
