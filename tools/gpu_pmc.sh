#!/bin/bash
# PMC passes over tools/kbench.py entries (KB, default the hot-path kernels at the bench shape):
# HBM traffic (FETCH_SIZE, WRITE_SIZE: one pass each) and VALU busy (SQ_ACTIVE_INST_VALU,
# SQ_INSTS_VALU, GRBM_GUI_ACTIVE), each pass its own run under `timeout -s KILL`, as the
# MI355X guide's rocprofv3 section prescribes.  Summaries: tools/pmc_traffic.py, tools/pmc_valu.py.
set -o pipefail
export TMPDIR=/tmp
ROOT=$GRAFT_REPO_ROOT
O=$ROOT/gpurun_out/${RUN_TAG:-pmc}
KB=${KB:-maps8,maps8_s16,maps8_s32,mapssel8,kl4}
mkdir -p $O
cd /tmp
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $c --kernel-trace -d $O/pmc_$c -o c --output-format csv -- python3 $ROOT/tools/kbench.py --only $KB --iters 3 > $O/pmc_$c.log 2>&1 || { echo "pmc $c failed"; tail -5 $O/pmc_$c.log; exit 12; }
done
timeout -s KILL 120 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_INSTS_VALU GRBM_GUI_ACTIVE --kernel-trace -d $O/pmc_valu -o c --output-format csv -- python3 $ROOT/tools/kbench.py --only $KB --iters 3 > $O/pmc_valu.log 2>&1 || { echo "pmc valu failed"; tail -5 $O/pmc_valu.log; exit 13; }
find $O -name "*counter_collection.csv"
echo pmc-ok
