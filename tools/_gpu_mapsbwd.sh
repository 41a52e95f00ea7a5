#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -v -s -p no:cacheprovider --timeout 300 --timeout-method thread -k "capture_maps or capture_bwd" > gpurun_out/mapsbwd_tests.log 2>&1 || { echo "tests failed rc=$?"; grep -E "Error|assert|FAILED" gpurun_out/mapsbwd_tests.log | head -20; tail -5 gpurun_out/mapsbwd_tests.log; exit 1; }
grep -E "passed|failed|fused" gpurun_out/mapsbwd_tests.log
timeout -k 10 180 python -u tools/kbench.py --only mapsbwd8,mapsbwd8_old,maps8 --iters 10 > gpurun_out/mapsbwd_kbench.log 2>&1 || { echo "kbench failed"; tail -20 gpurun_out/mapsbwd_kbench.log; exit 2; }
cat gpurun_out/mapsbwd_kbench.log
