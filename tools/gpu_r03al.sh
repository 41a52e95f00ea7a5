#!/bin/bash
# half-height Winograd blocks (32x16 px, 4 waves, two workgroups per CU; SKP_WINO2_HALF=1):
# conv tests vs fp64 with the variant on every TXB-8 shape, kernel timings A/B, bench A/B
set -o pipefail
export TMPDIR=/tmp
ROOT=$GRAFT_REPO_ROOT
O=$ROOT/gpurun_out/r03al
mkdir -p $O
cd $ROOT
SKP_WINO2_HALF=1 timeout -k 10 400 python -u -m pytest -x -q -p no:cacheprovider --timeout 120 --timeout-method thread tests/test_gpu_conv.py -m gpu > $O/tests.log 2>&1 || { echo "conv tests (half) failed"; grep -v amdgpu $O/tests.log | grep -v "^  File" | tail -25 | cut -c1-250; exit 1; }
tail -1 $O/tests.log
SH="8,128,128,512;8,256,256,256;8,512,512,128;8,512,512,64;8,320,320,64;8,640,640,32"
for v in 1 0 1 0; do
  SKP_WINO2_HALF=$v timeout -k 10 200 python -u tools/wino_time.py --shapes "$SH" > $O/wt_$v.log 2>&1 || { echo "wino_time failed"; tail -5 $O/wt_$v.log; exit 2; }
  SKP_WINO2_HALF=$v timeout -k 10 200 python -u tools/wino_time.py --residual --shapes "8,128,128,512" >> $O/wt_$v.log 2>&1 || { echo "wino_time failed"; exit 2; }
  echo "HALF=$v"; grep -v amdgpu $O/wt_$v.log
done
for v in 1 0 1 0; do
  SKP_WINO2_HALF=$v timeout -k 10 400 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline > $O/bench_$v.log 2>&1 || { echo "bench failed"; tail -5 $O/bench_$v.log; exit 3; }
  tail -1 $O/bench_$v.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('HALF=$v', round(d['value'],3), round(d['ms_per_step'],2))"
done
