#!/bin/bash
# r05zr: one-block-per-image top-k ranking (rank_topk_wide_kernel) vs the 16-lanes-per-key grid
set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/r05zr; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -k "topk or selection or entropy" --timeout 120 --timeout-method thread > $O/tests.log 2>&1; rc=$?; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
KB=kl4 RUN_TAG=r05zr ROUNDS=3 bash tools/gpu_kb_env.sh SKP_TOPK_WIDE=1 SKP_TOPK_WIDE=0 || exit 1
KB=kl4 RUN_TAG=r05zr_prof bash tools/gpu_kb_prof_env.sh SKP_TOPK_WIDE=1 SKP_TOPK_WIDE=0 || exit 1
echo r05zr-ok
