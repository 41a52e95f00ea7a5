#!/bin/bash
# r05v: fused A8 top-k with the coherence-point key handoff (tests, kbench kl4 fused vs separate,
# kernel durations), and FETCH_SIZE of the fused capture forward at 8- vs 16-wave workgroups (dev).
set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/r05v; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -k "topk or selection" --timeout 120 --timeout-method thread > $O/tests.log 2>&1; rc=$?; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
KB=kl4 RUN_TAG=r05v ROUNDS=2 bash tools/gpu_kb_env.sh SKP_TOPK_FUSED=1 SKP_TOPK_FUSED=0 || exit 1
KB=kl4 RUN_TAG=r05v_prof bash tools/gpu_kb_prof_env.sh SKP_TOPK_FUSED=1 SKP_TOPK_FUSED=0 || exit 1
cd /tmp
for w in 8 16; do
  SKP_MAPS_WAVES=$w timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $O/fetch_w$w -o c --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/kbench.py --only maps8 --iters 3 > $O/fetch_w$w.log 2>&1 || { echo "pmc w$w failed"; exit 12; }
done
echo r05v-ok
