#!/bin/bash
# split-K planner: half-height cost model (default) vs the r02 model (SKP_WINO_PLAN_HALF=0):
# UNet-shape conv timings and bench A/B; conv tests on the default
set -o pipefail
export TMPDIR=/tmp
ROOT=$GRAFT_REPO_ROOT
O=$ROOT/gpurun_out/r03an
mkdir -p $O
cd $ROOT
timeout -k 10 400 python -u -m pytest -x -q -p no:cacheprovider --timeout 120 --timeout-method thread tests/test_gpu_conv.py -m gpu > $O/tests.log 2>&1 || { echo "conv tests failed"; grep -v amdgpu $O/tests.log | tail -20; exit 1; }
tail -1 $O/tests.log
SH="8,320,320,64;8,640,640,32;8,320,640,32;8,1920,640,32;8,960,640,32;8,1280,320,32;8,640,320,64;8,1280,640,32"
for v in 1 0; do
  SKP_WINO_PLAN_HALF=$v timeout -k 10 200 python -u tools/wino_time.py --shapes "$SH" > $O/wt_$v.log 2>&1 || { echo "wino_time failed"; exit 2; }
  echo "PLAN_HALF=$v"; grep -v amdgpu $O/wt_$v.log
done
for v in 1 0 1 0; do
  SKP_WINO_PLAN_HALF=$v timeout -k 10 400 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline > $O/bench_$v.log 2>&1 || { echo "bench failed"; tail -5 $O/bench_$v.log; exit 3; }
  tail -1 $O/bench_$v.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('PLAN_HALF=$v', round(d['value'],3), round(d['ms_per_step'],2))"
done
