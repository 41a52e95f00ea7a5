#!/bin/bash
# the whole GPU suite (no -x: every failure is listed), one process, per-test timeout
set -o pipefail
export TMPDIR=/tmp
ROOT=$GRAFT_REPO_ROOT
O=$ROOT/gpurun_out/${RUN_TAG:-r03y}
mkdir -p $O
cd $ROOT
timeout -k 10 1000 python -u -m pytest tests -q -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread -rf > $O/gpu_tests.log 2>&1
rc=$?
tail -8 $O/gpu_tests.log
echo "rc=$rc"
