#!/bin/bash
# r05zi: streamed KL kernel with the window re-reads batched 4 per thread (tests + kernel time)
set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/r05zi; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -k "topk or selection or gaussian" --timeout 120 --timeout-method thread > $O/tests.log 2>&1; rc=$?; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
KB=kl4 RUN_TAG=r05zi_prof bash tools/gpu_kb_prof_env.sh SKP_KL_PROBE=0 SKP_KL_STREAM=0 || exit 1
echo r05zi-ok
