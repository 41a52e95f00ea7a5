#!/bin/bash
# GPU tests + bench + timed-region kernel profile, each step under its own limit; stops at the first failure.
set -o pipefail
R=${1:-r01}
mkdir -p gpurun_out
export TMPDIR=/tmp
ROOT=$GRAFT_REPO_ROOT
cd $ROOT
timeout -k 10 500 python -u -m pytest tests -x -v -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { echo "pytest failed rc=$?"; tail -40 gpurun_out/gpu_tests.log; exit 1; }
tail -2 gpurun_out/gpu_tests.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo "smoke failed"; tail -20 gpurun_out/smoke.log; exit 2; }
timeout -k 10 500 python -u bench.py > gpurun_out/bench.log 2>&1 || { echo "bench failed rc=$?"; tail -30 gpurun_out/bench.log; exit 3; }
tail -1 gpurun_out/bench.log
bash tools/gpu_prof_bench.sh $R || { echo "prof failed"; tail -20 gpurun_out/prof_$R.log; exit 4; }
echo all-ok
