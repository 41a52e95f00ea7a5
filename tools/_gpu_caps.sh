#!/bin/bash
# Fused capture fwd (two-row tile) + bwd (two heads per wave): parity of every form, then timing
set -o pipefail
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/caps
mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu -k "capture_maps or token_opt or batched" -p no:cacheprovider --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 120 python -u tools/kbench.py --only maps8,mapsbwd8 --iters 20 > $O/k_new.txt 2>&1 || { cat $O/k_new.txt; exit 2; }
SKP_MAPS_ROWS=1 SKP_BWD_HEADS=1 timeout -k 10 120 python -u tools/kbench.py --only maps8,mapsbwd8 --iters 20 > $O/k_old.txt 2>&1 || { cat $O/k_old.txt; exit 3; }
echo "new: $(grep maps $O/k_new.txt | tr '\n' ' ')"; echo "old: $(grep maps $O/k_old.txt | tr '\n' ' ')"
