#!/bin/bash
# r05zk: the 16-wave dual-job paired grid (build SKP_SEL_LW4=64) with compile-time LDS slices per
# half vs the default 8-wave grid: sparse-backward tests on the variant + same-box kbench (dev)
set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/r05zk; mkdir -p $O
SKP_LIB=$GRAFT_REPO_ROOT/build/var_lw64/libskp.so timeout -k 10 300 python -u -m pytest tests/test_gpu_sel_bwd.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1; rc=$?; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
KB=mapssel8 RUN_TAG=r05zk ROUNDS=3 bash tools/gpu_kb_env.sh SKP_NONE=1 SKP_LIB=$GRAFT_REPO_ROOT/build/var_lw64/libskp.so || exit 1
echo r05zk-ok
