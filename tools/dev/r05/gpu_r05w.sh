#!/bin/bash
# r05w: fused A8 top-k with the unrolled ranking tail (tests, kbench kl4 fused vs separate, kernel
# durations) and the fused capture forward at 8- vs 16-wave workgroups (kbench maps8) (dev script).
set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/r05w; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -k "topk or selection" --timeout 120 --timeout-method thread > $O/tests.log 2>&1; rc=$?; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
KB=kl4 RUN_TAG=r05w ROUNDS=2 bash tools/gpu_kb_env.sh SKP_TOPK_FUSED=1 SKP_TOPK_FUSED=0 || exit 1
KB=kl4 RUN_TAG=r05w_prof bash tools/gpu_kb_prof_env.sh SKP_TOPK_FUSED=1 || exit 1
KB=maps8 RUN_TAG=r05w_maps ROUNDS=3 KB_ITERS=30 bash tools/gpu_kb_env.sh SKP_MAPS_WAVES=8 SKP_MAPS_WAVES=16 || exit 1
echo r05w-ok
