# Winograd kernel diagnosis: timings with x / U loads dropped, then PMC passes on one shape.
set -o pipefail
export TMPDIR=/tmp
ROOT=$GRAFT_REPO_ROOT
mkdir -p $ROOT/gpurun_out/wdiag
cd $ROOT
for d in 0 1 2 3; do
  echo "dbg=$d"
  SKP_WINO_DEBUG=$d timeout -k 10 120 python -u tools/wino_time.py --shapes "8,128,128,512;8,512,512,64;8,320,320,64" || exit 9
done
cd /tmp
i=0
for set in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES" "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAIT_INST_LDS" "SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_INSTS_VALU SQ_INSTS_MFMA" "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_VMEM" "SQ_INSTS_SALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_FLAT SQ_WAVES"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $set --kernel-trace -d $ROOT/gpurun_out/wdiag/p$i -o c --output-format csv -- python $ROOT/tools/conv_one.py --iters 3 > $ROOT/gpurun_out/wdiag/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $ROOT/gpurun_out/wdiag/p$i.log; exit $i; }
done
echo done
