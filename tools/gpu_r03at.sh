#!/bin/bash
# head-major attention for the batch-shared context (SKP_SHARED_HEAD_MAJOR): tests, then bench
# A/Bs on the current tree — head-major on/off, and the VAE prefetch on a side stream (1) vs the
# main stream (0)
set -o pipefail
export TMPDIR=/tmp
ROOT=$GRAFT_REPO_ROOT
O=$ROOT/gpurun_out/r03at
mkdir -p $O
cd $ROOT
timeout -k 10 600 python -u -m pytest -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_attn_bshd.py tests/test_gpu_fullsize.py tests/test_gpu_graph.py > $O/tests.log 2>&1 || { echo "tests failed"; grep -v amdgpu $O/tests.log | grep -v "^  File" | tail -30 | cut -c1-250; exit 1; }
tail -1 $O/tests.log
run() {  # tag, env assignment, then bench args in BARGS
  local tag=$1; shift
  timeout -k 10 400 env "$@" python -u bench.py --steps 8 --warmup 3 --no-cpu-baseline $BARGS > $O/bench_$tag.log 2>&1 || { echo "bench $tag failed"; tail -5 $O/bench_$tag.log; return 4; }
  tail -1 $O/bench_$tag.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$tag', round(d['value'],3), round(d['ms_per_step'],2))"
}
for i in 1 2; do
  BARGS="--prefetch 1" run hm1_p1_$i SKP_SHARED_HEAD_MAJOR=1 || exit 4
  BARGS="--prefetch 1" run hm0_p1_$i SKP_SHARED_HEAD_MAJOR=0 || exit 4
  BARGS="--prefetch 0" run hm1_p0_$i SKP_SHARED_HEAD_MAJOR=1 || exit 4
done
