#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
ROOT=$GRAFT_REPO_ROOT
O=$ROOT/gpurun_out/r03g
mkdir -p $O
cd $ROOT
timeout -k 10 300 python -u tools/op_attrib.py --rows 30 > $O/op_attrib.log 2>&1 || { echo "op_attrib failed"; tail -20 $O/op_attrib.log; exit 1; }
grep -A45 "copy-like ops" $O/op_attrib.log | cut -c1-330
echo all-ok
