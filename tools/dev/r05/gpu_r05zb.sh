#!/bin/bash
# r05zb: streamed KL kernel, threads per row x float4 per chunk A/B (dev script)
set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/r05zb; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -k "topk or selection or gaussian" --timeout 120 --timeout-method thread > $O/tests.log 2>&1; rc=$?; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
KB=kl4 RUN_TAG=r05zb ROUNDS=3 bash tools/gpu_kb_env.sh "SKP_KL_BT=256 SKP_KL_UNR=2" "SKP_KL_BT=256 SKP_KL_UNR=1" "SKP_KL_BT=128 SKP_KL_UNR=2" "SKP_KL_BT=128 SKP_KL_UNR=1" "SKP_KL_BT=128 SKP_KL_UNR=4" || exit 1
echo r05zb-ok
