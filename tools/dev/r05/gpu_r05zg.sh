#!/bin/bash
# r05zg: the default build after the pair-grid generalisation: sparse-backward tests + kbench
set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/r05zg; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_sel_bwd.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1; rc=$?; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
KB=mapssel8,kl4,maps8 RUN_TAG=r05zg ROUNDS=2 bash tools/gpu_kb_env.sh SKP_NONE=1 || exit 1
echo r05zg-ok
