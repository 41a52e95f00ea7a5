#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
ROOT=$GRAFT_REPO_ROOT
O=$ROOT/gpurun_out/r03u
mkdir -p $O
cd $ROOT
timeout -k 10 300 python -u tools/copy_sites.py --rows 80 > $O/copy_sites.log 2>&1 || { echo "copy_sites failed rc=$?"; grep -v amdgpu $O/copy_sites.log | tail -20 | cut -c1-300; exit 1; }
grep -v amdgpu $O/copy_sites.log | head -50 | cut -c1-250
