# conv tests, then Winograd timings (v1, v2, v2 switches)
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_conv.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/conv_tests.log 2>&1; rc=$?
tail -3 gpurun_out/conv_tests.log
[ $rc -eq 0 ] || { tail -40 gpurun_out/conv_tests.log; exit $rc; }
echo "v1"; SKP_WINO=v1 timeout -k 10 120 python -u tools/wino_time.py || exit 9
echo "v2"; timeout -k 10 120 python -u tools/wino_time.py || exit 9
for d in ${DBGS:-}; do echo "v2 dbg=$d"; SKP_WINO2_DEBUG=$d timeout -k 10 120 python -u tools/wino_time.py --shapes "8,128,128,512;8,512,512,64" || exit 9; done
