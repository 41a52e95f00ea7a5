#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
ROOT=$GRAFT_REPO_ROOT
O=$ROOT/gpurun_out/r03o
mkdir -p $O
cd $ROOT
timeout -k 10 400 python -u tools/host_profile.py --rows 45 > $O/hp.log 2>&1 || { echo "host_profile failed"; tail -20 $O/hp.log; exit 1; }
grep -v amdgpu $O/hp.log | head -70 | cut -c1-200
echo all-ok
