#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
ROOT=$GRAFT_REPO_ROOT
O=$ROOT/gpurun_out/r03r
mkdir -p $O
cd $ROOT
timeout -k 10 300 python -u tools/prefetch_time2.py > $O/pt.log 2>&1 || { echo "prefetch_time failed"; tail -20 $O/pt.log; exit 1; }
grep prefetch $O/pt.log
echo all-ok
