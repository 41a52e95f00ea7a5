#!/bin/bash
# r05zl: sel_doth variants vs HEAD's build (libskp_base.so): tests, same-box kbench, per-kernel profile (dev script)
set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/${TAG:-r05zl}; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_sel_bwd.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1; rc=$?; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
KB=mapssel8 RUN_TAG=${TAG:-r05zl} ROUNDS=3 bash tools/gpu_kb_env.sh SKP_NONE=1 SKP_LIB=$GRAFT_REPO_ROOT/stablekeypoints_amd/libskp_base.so || exit 1
KB=mapssel8 RUN_TAG=${TAG:-r05zl}_prof bash tools/gpu_kb_prof_env.sh SKP_NONE=1 || exit 1
echo r05zl-ok
