#!/bin/bash
# Same-box A/B of libskp.so builds (dev tool): optionally the GPU tests TESTS (pytest arguments) on
# the working tree, then rocprofv3 kernel stats of the kbench entries KB for each library in LIBS
# ("tree" = the in-tree build; otherwise a path under the repo, e.g. stablekeypoints_amd/libskp_base.so
# from tools/build_rev.sh or build/var_NAME/libskp.so from tools/build_variant.sh), ROUNDS times.
#   TESTS="tests/test_gpu_sel_bwd.py" KB=mapssel8 LIBS="stablekeypoints_amd/libskp_base.so tree" bash tools/gpu_kb_ab.sh
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/${RUN_TAG:-kbab}
mkdir -p $O
cd $GRAFT_REPO_ROOT
if [ -n "$TESTS" ]; then
  timeout -k 10 400 python -u -m pytest $TESTS -x -q -p no:cacheprovider --timeout 150 --timeout-method thread > $O/t.log 2>&1 || { echo "tests failed"; tail -30 $O/t.log; exit 1; }
  tail -1 $O/t.log
fi
args=()
for r in $(seq 1 ${ROUNDS:-2}); do
  for l in ${LIBS:-tree}; do
    if [ "$l" = tree ]; then args+=("SKP_NONE=1"); else args+=("SKP_LIB=$GRAFT_REPO_ROOT/$l"); fi
  done
done
RUN_TAG=${RUN_TAG:-kbab}/prof bash tools/gpu_kb_prof_env.sh "${args[@]}"
