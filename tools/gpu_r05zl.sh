#!/bin/bash
# r05zl: sel_doth with 16-B / 8-B LDS reads in its column filters vs HEAD's build (dev script)
set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/r05zl; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_sel_bwd.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1; rc=$?; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
KB=mapssel8 RUN_TAG=r05zl ROUNDS=3 bash tools/gpu_kb_env.sh SKP_NONE=1 SKP_LIB=$GRAFT_REPO_ROOT/stablekeypoints_amd/libskp_base.so || exit 1
KB=mapssel8 RUN_TAG=r05zl_prof bash tools/gpu_kb_prof_env.sh SKP_NONE=1 || exit 1
echo r05zl-ok
