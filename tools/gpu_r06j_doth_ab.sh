# r06 sel_doth A/B (dev): the sparse-backward GPU tests on the working tree and on the variant
# libraries, then rocprofv3 kernel stats of kbench mapssel8 for HEAD's library (libskp_base.so),
# the tree's and the variants
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/${RUN_TAG:-r06j}; mkdir -p $O; cd $GRAFT_REPO_ROOT
R=/root/repo
timeout -k 10 300 python -u -m pytest tests/test_gpu_sel_bwd.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $O/t.log 2>&1 || { echo "tests failed"; tail -30 $O/t.log; exit 1; }
tail -1 $O/t.log
for v in ${VARIANTS:-}; do
  SKP_LIB=$R/build/var_$v/libskp.so timeout -k 10 300 python -u -m pytest tests/test_gpu_sel_bwd.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $O/t_$v.log 2>&1 || { echo "tests ($v) failed"; tail -30 $O/t_$v.log; exit 1; }
  echo "$v: $(tail -1 $O/t_$v.log)"
done
args=("SKP_LIB=$R/stablekeypoints_amd/libskp_base.so" "SKP_NONE=1")
for v in ${VARIANTS:-}; do args+=("SKP_LIB=$R/build/var_$v/libskp.so"); done
args+=("SKP_NONE=1")
KB=mapssel8 bash tools/gpu_kb_prof_env.sh "${args[@]}"
