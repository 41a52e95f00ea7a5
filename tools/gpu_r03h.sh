#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
ROOT=$GRAFT_REPO_ROOT
O=$ROOT/gpurun_out/r03h
mkdir -p $O
cd $ROOT
timeout -k 10 500 python -u -m pytest -x -q -p no:cacheprovider --timeout 120 --timeout-method thread tests/test_gpu_conv.py -m gpu > $O/tests.log 2>&1 || { echo "tests failed rc=$?"; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 200 python -u tools/conv_s2_time.py > $O/conv_s2.log 2>&1 || { echo "conv_s2 failed"; tail -20 $O/conv_s2.log; exit 2; }
grep -v amdgpu $O/conv_s2.log
for v in 1 0 1 0; do
  SKP_WINO_S2=$v SKP_CONV1X1_GEMM=$v timeout -k 10 400 python -u bench.py --no-cpu-baseline --steps 4 > $O/bench_$v.log 2>&1 || { echo "bench $v failed"; tail -20 $O/bench_$v.log; exit 3; }
  echo "S2+1x1=$v $(tail -1 $O/bench_$v.log | cut -c1-150)"
done
SKP_CONV1X1_GEMM=0 timeout -k 10 400 python -u bench.py --no-cpu-baseline --steps 4 > $O/bench_s2only.log 2>&1 || { echo "bench s2only failed"; exit 4; }
echo "S2 only $(tail -1 $O/bench_s2only.log | cut -c1-150)"
echo all-ok
