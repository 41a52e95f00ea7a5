#!/bin/bash
# wino2 raw-input ring of 4 slots (lead 3) vs 3: conv parity, then timing
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/w2rs
mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_conv.py -x -q -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
SH="8,128,128,512;8,512,512,64;8,320,320,64;8,640,640,32;8,256,256,256;8,512,512,128;8,1280,1280,16"
for i in 1 2; do
echo "== rs4"; timeout -k 10 120 python -u tools/wino_time.py --shapes "$SH" || exit 2
echo "== rs3"; SKP_LIB=build/var_rs3/libskp.so timeout -k 10 120 python -u tools/wino_time.py --shapes "$SH" || exit 3
done
