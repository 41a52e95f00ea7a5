#!/bin/bash
# Winograd as transforms + 36 batched library GEMMs for the UNet's small-image convolutions:
# conv tests, per-shape timings (SKP_WINO_GEMM_MAX_HW 0 = fused kernels vs GEMM form), bench A/B
set -o pipefail
export TMPDIR=/tmp
ROOT=$GRAFT_REPO_ROOT
O=$ROOT/gpurun_out/r03ax
mkdir -p $O
cd $ROOT
timeout -k 10 500 python -u -m pytest -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_conv.py > $O/tests.log 2>&1 || { echo "conv tests failed"; grep -v amdgpu $O/tests.log | grep -v "^  File" | tail -30 | cut -c1-250; exit 1; }
tail -1 $O/tests.log
SH="8,1280,1280,16;8,2560,1280,16;8,1920,1280,16;8,1280,1280,8;8,2560,1280,8;8,640,640,32;8,1280,640,32;8,960,640,32;8,320,320,64;8,640,320,64"
for v in 0 4096; do
  SKP_WINO_GEMM_MAX_HW=$v timeout -k 10 200 python -u tools/wino_time.py --shapes "$SH" --residual > $O/wt_$v.log 2>&1 || { echo "wino_time failed"; tail -5 $O/wt_$v.log; exit 2; }
  echo "MAX_HW=$v"; grep -v amdgpu $O/wt_$v.log
done
for v in 1024 0 256 1024 0 4096; do
  SKP_WINO_GEMM_MAX_HW=$v timeout -k 10 400 python -u bench.py --steps 8 --warmup 3 --no-cpu-baseline > $O/bench_$v.log 2>&1 || { echo "bench failed"; tail -5 $O/bench_$v.log; exit 4; }
  tail -1 $O/bench_$v.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('MAX_HW=$v', round(d['value'],3), round(d['ms_per_step'],2))"
done
