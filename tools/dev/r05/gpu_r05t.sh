#!/bin/bash
# r05t: sel_doth as per-virtual-column dot products (registers bounded per launch class): sparse
# backward tests, kbench A/B against the E path, per-kernel profile (dev script).
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r05t; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_sel_bwd.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1; rc=$?; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
KB=mapssel8 RUN_TAG=r05t ROUNDS=3 bash tools/gpu_kb_env.sh SKP_SEL_DOTH=0 SKP_SEL_DOTH=1 || exit 1
KB=mapssel8 RUN_TAG=r05t_prof bash tools/gpu_kb_prof_env.sh SKP_SEL_DOTH=1 SKP_SEL_DOTH=0 || exit 1
