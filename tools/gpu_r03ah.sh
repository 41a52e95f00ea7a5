#!/bin/bash
# Winograd non-temporal output stores: conv tests with the NT path forced on every shape, conv
# timings and bench A/B (SKP_WINO_NT 0 vs default), then the capture-forward PMC refresh
set -o pipefail
export TMPDIR=/tmp
ROOT=$GRAFT_REPO_ROOT
O=$ROOT/gpurun_out/r03ah
mkdir -p $O
cd $ROOT
SKP_WINO_NT=2 timeout -k 10 400 python -u -m pytest -x -q -p no:cacheprovider --timeout 120 --timeout-method thread tests/test_gpu_conv.py -m gpu > $O/tests.log 2>&1 || { echo "conv tests (NT forced) failed"; grep -v amdgpu $O/tests.log | tail -20; exit 1; }
tail -1 $O/tests.log
for v in 1 0 1 0; do
  SKP_WINO_NT=$v timeout -k 10 200 python -u tools/wino_time.py --shapes "8,128,128,512;8,256,256,256;8,512,512,128" > $O/wt_$v.log 2>&1 || { echo "wino_time failed"; tail -5 $O/wt_$v.log; exit 2; }
  SKP_WINO_NT=$v timeout -k 10 200 python -u tools/wino_time.py --residual --shapes "8,128,128,512" >> $O/wt_$v.log 2>&1 || { echo "wino_time failed"; exit 2; }
  echo "NT=$v"; grep -v amdgpu $O/wt_$v.log
done
for v in 0 1 0 1; do
  SKP_WINO_NT=$v timeout -k 10 400 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline > $O/bench_$v.log 2>&1 || { echo "bench failed"; tail -5 $O/bench_$v.log; exit 3; }
  tail -1 $O/bench_$v.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('NT=$v', round(d['value'],3), round(d['ms_per_step'],2))"
done
bash tools/gpu_r03ag.sh
