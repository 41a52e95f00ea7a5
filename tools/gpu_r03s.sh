#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
ROOT=$GRAFT_REPO_ROOT
O=$ROOT/gpurun_out/r03s
mkdir -p $O
cd $ROOT
timeout -k 10 400 python -u tools/graph_try.py > $O/g.log 2>&1; rc=$?
grep -v amdgpu $O/g.log | tail -30 | cut -c1-400
echo "rc=$rc"
