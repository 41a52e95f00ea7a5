#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
ROOT=$GRAFT_REPO_ROOT
O=$ROOT/gpurun_out/r03n
mkdir -p $O
cd $ROOT
HOST_ORDER=after timeout -k 10 400 python -u tools/host_time.py > $O/host.log 2>&1 || { echo "host_time failed"; tail -20 $O/host.log; exit 1; }
grep -v amdgpu $O/host.log | tail -4
for i in 1 2; do
  timeout -k 10 400 python -u bench.py --no-cpu-baseline --steps 8 > $O/bench_$i.log 2>&1 || { echo "bench failed"; tail -20 $O/bench_$i.log; exit 3; }
  echo "bench $(tail -1 $O/bench_$i.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["value"],2), round(d["ms_per_step"],2))')"
done
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace -d $O/prof -o bench --output-format csv -- python3 $ROOT/bench.py --steps 2 --warmup 2 --no-cpu-baseline > $O/prof.log 2>&1 || { echo "prof failed"; tail -5 $O/prof.log; exit 1; }
cd $ROOT && python3 tools/stream_gaps.py $O/prof/bench_kernel_trace.csv --top 6
timeout -k 10 700 python -u -m pytest tests -x -q -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo "pytest failed rc=$?"; tail -30 $O/gpu_tests.log; exit 4; }
tail -1 $O/gpu_tests.log
echo all-ok
