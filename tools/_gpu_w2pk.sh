#!/bin/bash
# packed Winograd input transform: conv parity, then timing vs the scalar-transform build
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/w2pk
mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_conv.py -x -q -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
SH="8,128,128,512;8,512,512,64;8,320,320,64;8,640,640,32;8,256,256,256"
for i in 1 2; do
echo "== packed"; timeout -k 10 120 python -u tools/wino_time.py --shapes "$SH" || exit 2
echo "== scalar"; SKP_LIB=build/var_w2old/libskp.so timeout -k 10 120 python -u tools/wino_time.py --shapes "$SH" || exit 3
done
