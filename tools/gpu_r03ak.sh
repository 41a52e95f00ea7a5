#!/bin/bash
# fused capture forward: 16-wave workgroups vs 8 on the persistent / non-temporal build (kbench A/B)
set -o pipefail
export TMPDIR=/tmp
ROOT=$GRAFT_REPO_ROOT
O=$ROOT/gpurun_out/r03ak
mkdir -p $O
cd $ROOT
for w in 16 8 16 8; do
  SKP_MAPS_WAVES=$w timeout -k 10 200 python -u tools/kbench.py --only maps8 --iters 20 > $O/kb_$w.log 2>&1 || { echo "kbench failed"; exit 2; }
  echo "waves=$w $(grep maps8 $O/kb_$w.log)"
done
