#!/bin/bash
# split-K sweep of the UNet's 64² / 32² Winograd shapes on the half-height default (SKP_WINO_NSPLIT)
set -o pipefail
export TMPDIR=/tmp
ROOT=$GRAFT_REPO_ROOT
O=$ROOT/gpurun_out/r03am
mkdir -p $O
cd $ROOT
for S in 0 1 2 4 5 8 10; do
  SKP_WINO_NSPLIT=$S timeout -k 10 200 python -u tools/wino_time.py --shapes "8,320,320,64;8,640,640,32;8,320,640,32;8,1920,640,32;8,960,640,32" > $O/s_$S.log 2>&1 || { echo "failed S=$S"; tail -5 $O/s_$S.log; exit 1; }
  echo "S=$S"; grep -v amdgpu $O/s_$S.log
done
