# PMC passes for the capture backward (rows + cols kernels) at the bench's per-image shapes
set -o pipefail
export TMPDIR=/tmp
ROOT=$GRAFT_REPO_ROOT
mkdir -p $ROOT/gpurun_out/pmccap
cd /tmp
i=0
for set in "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE" "SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_WAIT_ANY" "SQ_INSTS_VALU_TRANS_F32 SQ_ACTIVE_INST_LDS SQ_BUSY_CYCLES SQ_WAVES"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $set --kernel-trace -d $ROOT/gpurun_out/pmccap/p$i -o c --output-format csv -- python $ROOT/tools/kbench.py --only bwd16b2 --iters 3 > $ROOT/gpurun_out/pmccap/p$i.log 2>&1 || { echo "pass $i failed"; tail -3 $ROOT/gpurun_out/pmccap/p$i.log; }
done
echo done
