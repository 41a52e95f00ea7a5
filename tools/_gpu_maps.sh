#!/bin/bash
# Fused capture+aggregate: parity tests, then micro-bench (fused vs two-kernel) and its kernel trace.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -v -s -p no:cacheprovider --timeout 200 --timeout-method thread -k "capture_maps or capture_bwd_with" > gpurun_out/maps_tests.log 2>&1 || { echo "tests failed rc=$?"; tail -40 gpurun_out/maps_tests.log; exit 1; }
grep -E "passed|failed|fused vs" gpurun_out/maps_tests.log
timeout -k 10 120 python -u tools/kbench.py --only maps8,maps8_old --iters 10 > gpurun_out/maps_kbench.log 2>&1 || { echo "kbench failed"; tail -20 gpurun_out/maps_kbench.log; exit 2; }
cat gpurun_out/maps_kbench.log
cd /tmp && timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_maps -o maps --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/kbench.py --only maps8 --iters 5 > $GRAFT_REPO_ROOT/gpurun_out/prof_maps.log 2>&1 || { echo "prof failed"; exit 3; }
cd $GRAFT_REPO_ROOT; f=$(find gpurun_out/prof_maps -name "*kernel_stats.csv" | head -1); cut -d, -f1-8 "$f" | head -6
echo all-ok
