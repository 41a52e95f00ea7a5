#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
ROOT=$GRAFT_REPO_ROOT
O=$ROOT/gpurun_out/r03q
mkdir -p $O
cd $ROOT
timeout -k 10 400 python -u tools/host_time.py --prefetch 1 > $O/host.log 2>&1 || { echo "host_time failed"; tail -20 $O/host.log; exit 1; }
grep -v amdgpu $O/host.log | tail -3
for p in 1 2 1 2; do
  timeout -k 10 400 python -u bench.py --no-cpu-baseline --steps 8 --prefetch $p > $O/bench_$p.log 2>&1 || { echo "bench failed"; tail -20 $O/bench_$p.log; exit 3; }
  echo "prefetch $p: $(tail -1 $O/bench_$p.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["value"],2), round(d["ms_per_step"],2))')"
done
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace -d $O/prof -o bench --output-format csv -- python3 $ROOT/bench.py --steps 2 --warmup 2 --no-cpu-baseline > $O/prof.log 2>&1 || { echo "prof failed"; tail -5 $O/prof.log; exit 1; }
cd $ROOT && python3 tools/stream_gaps.py $O/prof/bench_kernel_trace.csv --top 6
echo all-ok
