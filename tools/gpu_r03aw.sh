#!/bin/bash
# batched selection + batched losses (SKP_SEL_BATCH): parity tests, then bench A/B
# parity tests, the step tests, then bench A/B SKP_SEL_BATCH=1 vs 0 (alternating)
set -o pipefail
export TMPDIR=/tmp
ROOT=$GRAFT_REPO_ROOT
O=$ROOT/gpurun_out/r03aw
mkdir -p $O
cd $ROOT
timeout -k 10 600 python -u -m pytest -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py tests/test_gpu_graph.py tests/test_gpu_sel_bwd.py tests/test_gpu_configs.py tests/test_gpu_refapi.py > $O/tests.log 2>&1 || { echo "tests failed"; grep -v amdgpu $O/tests.log | grep -v "^  File" | tail -30 | cut -c1-250; exit 1; }
tail -1 $O/tests.log
for v in 1 0 1 0; do
  SKP_SEL_BATCH=$v timeout -k 10 400 python -u bench.py --steps 8 --warmup 3 --no-cpu-baseline > $O/bench_$v.log 2>&1 || { echo "bench failed"; tail -5 $O/bench_$v.log; exit 4; }
  tail -1 $O/bench_$v.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('SEL_BATCH=$v', round(d['value'],3), round(d['ms_per_step'],2))"
done
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof -o bench --output-format csv -- python3 $ROOT/bench.py --steps 2 --warmup 2 --no-cpu-baseline > $O/prof.log 2>&1 || { echo "prof failed"; tail -5 $O/prof.log; exit 9; }
cd $ROOT && python3 tools/prof_summary.py $O/prof/bench_kernel_trace.csv --steps 2 --accum 4 --out $O/timed_summary.csv --top 60 > $O/timed_summary.txt
