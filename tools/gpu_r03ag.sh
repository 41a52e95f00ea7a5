#!/bin/bash
# PMC records of the fused capture forward on the current default build (persistent grid,
# non-temporal map/stats stores): FETCH_SIZE, WRITE_SIZE, VALU passes on kbench maps8 / _s16 / _s32
set -o pipefail
export TMPDIR=/tmp
ROOT=$GRAFT_REPO_ROOT
O=$ROOT/gpurun_out/r03ag
mkdir -p $O
cd /tmp
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $c --kernel-trace -d $O/pmc_$c -o c --output-format csv -- python3 $ROOT/tools/kbench.py --only maps8,maps8_s16,maps8_s32 --iters 3 > $O/pmc_$c.log 2>&1 || { echo "pmc $c failed"; exit 1; }
done
timeout -s KILL 120 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_INSTS_VALU GRBM_GUI_ACTIVE --kernel-trace -d $O/pmc_valu -o c --output-format csv -- python3 $ROOT/tools/kbench.py --only maps8 --iters 3 > $O/pmc_valu.log 2>&1 || { echo "pmc valu failed"; exit 2; }
cd $ROOT
timeout -k 10 200 python -u tools/kbench.py --only maps8,maps8_s16,maps8_s32,mapssel8 --iters 20 > $O/kbench.log 2>&1 || { echo "kbench failed"; exit 3; }
grep -v amdgpu $O/kbench.log
echo ok
