# PMC clock / MFMA-busy for skp_conv3x3_wino2 on one shape under debug switches
set -o pipefail
export TMPDIR=/tmp
ROOT=$GRAFT_REPO_ROOT
mkdir -p $ROOT/gpurun_out/w2pmc
cd /tmp
for d in 0 1 2; do
  SKP_WINO2_DEBUG=$d timeout -s KILL 90 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA --kernel-trace -d $ROOT/gpurun_out/w2pmc/d$d -o c --output-format csv -- python $ROOT/tools/conv_one.py --shape ${SHAPE:-8,128,128,512} --iters 4 > $ROOT/gpurun_out/w2pmc/d$d.log 2>&1 || { echo "pass $d failed"; tail -5 $ROOT/gpurun_out/w2pmc/d$d.log; exit 1; }
done
echo done
