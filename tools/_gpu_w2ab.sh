#!/bin/bash
# wino2 A/B: conv parity on the default build, then timing vs build/var_$VAR
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out/w2ab
mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_conv.py -x -q -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
SH="8,128,128,512;8,512,512,64;8,320,320,64;8,640,640,32;8,256,256,256;8,512,512,128;8,1280,1280,16"
for i in 1 2; do
echo "== default"; timeout -k 10 120 python -u tools/wino_time.py --shapes "$SH" || exit 2
echo "== $VAR"; SKP_LIB=build/var_$VAR/libskp.so timeout -k 10 120 python -u tools/wino_time.py --shapes "$SH" || exit 3
done
