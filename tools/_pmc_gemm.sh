#!/bin/bash
# PMC pass over the bgemm micro-benchmark: MFMA busy, waits, LDS conflicts
set -o pipefail
export TMPDIR=/tmp
ROOT=$GRAFT_REPO_ROOT
OUT=$ROOT/gpurun_out/pmc_gemm
mkdir -p $OUT
cd /tmp
timeout -s KILL 90 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS GRBM_GUI_ACTIVE --kernel-trace -d $OUT/p1 -o c --output-format csv -- python3 $ROOT/tools/kbench.py --only gemm16 --iters 3 > $OUT/p1.log 2>&1 || { echo "pass failed"; tail -3 $OUT/p1.log; exit 1; }
cd $ROOT && python3 tools/pmc_summary.py $OUT --match bgemm
