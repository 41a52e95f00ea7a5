#!/bin/bash
# capture forward, producer-wave form: bit-exact A/B test + oracle parity, then kernel timings A/B
set -o pipefail
export TMPDIR=/tmp
ROOT=$GRAFT_REPO_ROOT
O=$ROOT/gpurun_out/r03v
mkdir -p $O
cd $ROOT
PT="python -u -m pytest -x -v -p no:cacheprovider --timeout 120 --timeout-method thread"
timeout -k 10 300 $PT tests/test_gpu_parity.py -m gpu -k "capture_maps" > $O/tests.log 2>&1 || { echo "tests failed rc=$?"; grep -v amdgpu $O/tests.log | grep -v "^  File" | tail -30 | cut -c1-300; exit 1; }
tail -1 $O/tests.log
for w in 1 0 1 0; do
  SKP_MAPS_WS=$w timeout -k 10 200 python -u tools/kbench.py --only maps8 --iters 20 > $O/kb_$w.log 2>&1 || { echo "kbench $w failed"; tail -20 $O/kb_$w.log; exit 2; }
  echo "ws=$w"; grep -v amdgpu $O/kb_$w.log | tail -3
done
