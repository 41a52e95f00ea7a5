#!/bin/bash
# r05s: sparse-backward changes (sel_doth / sel_adjv, |d| folded into sel_dense's exponent) and the
# flattened Winograd transform grids: tests, kbench A/Bs, per-kernel profile, bench A/B vs HEAD's
# library, and the r04c regression re-run on the two commits around it (dev script).
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r05s; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_sel_bwd.py tests/test_gpu_conv.py tests/test_gpu_gn_epi.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1; rc=$?; tail -3 $O/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q -k "topk or selection or entropy" --timeout 120 --timeout-method thread > $O/tests2.log 2>&1; rc=$?; tail -3 $O/tests2.log; [ $rc -eq 0 ] || exit $rc
KB=mapssel8 RUN_TAG=r05s ROUNDS=3 bash tools/gpu_kb_env.sh SKP_SEL_DOTH=0 SKP_SEL_DOTH=1 SKP_LIB=$GRAFT_REPO_ROOT/build/var_nofold/libskp.so || exit 1
KB=mapssel8 RUN_TAG=r05s_prof bash tools/gpu_kb_prof_env.sh SKP_SEL_DOTH=1 || exit 1
RUN_TAG=r05s_ab ROUNDS=2 ARGS="--steps 10 --warmup 3" bash tools/gpu_ab_env.sh SKP_LIB=$GRAFT_REPO_ROOT/stablekeypoints_amd/libskp_base.so SKP_NONE=1 || exit 1
for r in 46add6f e1869ea; do (cd build/rev_$r && timeout -k 10 240 python -u -m pytest tests/test_gpu_parity.py -q -k "micro_steps_batch_equals_sequential" --timeout 200 --timeout-method thread > $GRAFT_REPO_ROOT/$O/repro_$r.log 2>&1; echo "$r rc=$?"; tail -2 $GRAFT_REPO_ROOT/$O/repro_$r.log); done
