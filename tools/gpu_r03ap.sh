#!/bin/bash
# 16×16 Winograd geometry, 4-wave form (two images per workgroup, two workgroups per CU;
# SKP_WINO2_HALF16=1): conv tests, timings and bench A/B
set -o pipefail
export TMPDIR=/tmp
ROOT=$GRAFT_REPO_ROOT
O=$ROOT/gpurun_out/r03ap
mkdir -p $O
cd $ROOT
SKP_WINO2_HALF16=1 timeout -k 10 400 python -u -m pytest -x -q -p no:cacheprovider --timeout 120 --timeout-method thread tests/test_gpu_conv.py -m gpu > $O/tests.log 2>&1 || { echo "conv tests failed"; grep -v amdgpu $O/tests.log | grep -v "^  File" | tail -25 | cut -c1-250; exit 1; }
tail -1 $O/tests.log
SH="8,1280,1280,16;8,2560,1280,16;8,640,1280,16;8,1920,1280,16;8,1280,640,16"
for v in 1 0 1 0; do
  SKP_WINO2_HALF16=$v timeout -k 10 200 python -u tools/wino_time.py --shapes "$SH" > $O/wt_$v.log 2>&1 || { echo "wino_time failed"; tail -5 $O/wt_$v.log; exit 2; }
  echo "HALF16=$v"; grep -v amdgpu $O/wt_$v.log
done
for S in 2 4 8 16; do
  SKP_WINO2_HALF16=1 SKP_WINO_NSPLIT=$S timeout -k 10 200 python -u tools/wino_time.py --shapes "$SH" > $O/ws_$S.log 2>&1 || { echo "split failed"; exit 3; }
  echo "HALF16=1 S=$S"; grep -v amdgpu $O/ws_$S.log
done
for v in 1 0 1 0; do
  SKP_WINO2_HALF16=$v timeout -k 10 400 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline > $O/bench_$v.log 2>&1 || { echo "bench failed"; tail -5 $O/bench_$v.log; exit 4; }
  tail -1 $O/bench_$v.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('HALF16=$v', round(d['value'],3), round(d['ms_per_step'],2))"
done
