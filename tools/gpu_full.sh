#!/bin/bash
# Full-size production-path parity test (printed numbers), then the GPU suite and the default bench.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests/test_gpu_fullsize.py -x -v -s -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/fullsize.log 2>&1 || { echo "fullsize failed rc=$?"; tail -40 gpurun_out/fullsize.log; exit 1; }
grep -E "full-size|capture_sd15|passed|failed" gpurun_out/fullsize.log
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread --deselect tests/test_gpu_fullsize.py > gpurun_out/gpu_tests.log 2>&1 || { echo "pytest failed rc=$?"; tail -40 gpurun_out/gpu_tests.log; exit 2; }
tail -2 gpurun_out/gpu_tests.log
timeout -k 10 500 python -u bench.py > gpurun_out/bench.log 2>&1 || { echo "bench failed rc=$?"; tail -30 gpurun_out/bench.log; exit 3; }
tail -1 gpurun_out/bench.log
echo all-ok
