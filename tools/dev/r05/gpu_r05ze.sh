#!/bin/bash
# r05ze: sel_dense at R/s = 4 with whole-wave bands (16-wave blocks, separate class launches) vs
# the default half-wave bands in the paired grid, and the unpaired default (dev script)
set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/r05ze; mkdir -p $O
SKP_LIB=$GRAFT_REPO_ROOT/build/var_lw64/libskp.so timeout -k 10 300 python -u -m pytest tests/test_gpu_sel_bwd.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1; rc=$?; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
KB=mapssel8,mapssel8_s16,mapssel8_s32 RUN_TAG=r05ze ROUNDS=2 bash tools/gpu_kb_env.sh SKP_NONE=1 SKP_LIB=$GRAFT_REPO_ROOT/build/var_nopair/libskp.so SKP_LIB=$GRAFT_REPO_ROOT/build/var_lw64/libskp.so || exit 1
KB=mapssel8_s32 RUN_TAG=r05ze_prof bash tools/gpu_kb_prof_env.sh SKP_NONE=1 SKP_LIB=$GRAFT_REPO_ROOT/build/var_lw64/libskp.so || exit 1
echo r05ze-ok
