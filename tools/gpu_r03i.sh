#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
ROOT=$GRAFT_REPO_ROOT
O=$ROOT/gpurun_out/r03i
mkdir -p $O
cd $ROOT
timeout -k 10 500 python -u -m pytest -x -q -p no:cacheprovider --timeout 120 --timeout-method thread tests/test_gpu_conv.py -m gpu -k "stride2 or conv1x1 or resnet or downsample" > $O/tests.log 2>&1 || { echo "tests failed rc=$?"; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 200 python -u tools/conv1x1_time.py > $O/c11.log 2>&1 || { echo "c11 failed"; tail -20 $O/c11.log; exit 2; }
grep -v amdgpu $O/c11.log
for v in 1 0 1 0; do
  SKP_CONV1X1_GEMM=$v timeout -k 10 400 python -u bench.py --no-cpu-baseline --steps 8 > $O/bench_$v.log 2>&1 || { echo "bench $v failed"; tail -20 $O/bench_$v.log; exit 3; }
  echo "1x1GEMM=$v $(tail -1 $O/bench_$v.log | cut -c90-140)"
done
echo all-ok
