#!/bin/bash
# r05za: streamed KL kernel without the separate block max, chunk size A/B (dev script)
set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/r05za; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -k "topk or selection or gaussian" --timeout 120 --timeout-method thread > $O/tests.log 2>&1; rc=$?; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
KB=kl4 RUN_TAG=r05za ROUNDS=3 bash tools/gpu_kb_env.sh SKP_KL_UNR=4 SKP_KL_UNR=2 SKP_KL_UNR=8 SKP_KL_STREAM=0 || exit 1
KB=kl4 RUN_TAG=r05za_prof bash tools/gpu_kb_prof_env.sh SKP_KL_UNR=4 SKP_KL_UNR=8 || exit 1
echo r05za-ok
