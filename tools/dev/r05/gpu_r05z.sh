#!/bin/bash
# r05z: streamed KL ranking kernel (tests, kbench kl4 A/B against the held form, kernel durations)
set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/r05z; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_eval.py -x -q -k "topk or selection or gaussian or find_best" --timeout 120 --timeout-method thread > $O/tests.log 2>&1; rc=$?; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
KB=kl4 RUN_TAG=r05z ROUNDS=3 bash tools/gpu_kb_env.sh SKP_KL_STREAM=1 SKP_KL_STREAM=0 || exit 1
KB=kl4 RUN_TAG=r05z_prof bash tools/gpu_kb_prof_env.sh SKP_KL_STREAM=1 SKP_KL_STREAM=0 || exit 1
echo r05z-ok
KB=mapssel8_s16,mapssel8_s32 RUN_TAG=r05z_cls bash tools/gpu_kb_prof_env.sh SKP_NONE=1 || exit 1
