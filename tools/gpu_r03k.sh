#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
ROOT=$GRAFT_REPO_ROOT
O=$ROOT/gpurun_out/r03k
mkdir -p $O
cd $ROOT
for p in 2 1 2 1; do
  timeout -k 10 400 python -u bench.py --no-cpu-baseline --steps 8 --prefetch $p > $O/bench_p$p.log 2>&1 || { echo "bench $p failed"; tail -20 $O/bench_p$p.log; exit 3; }
  echo "prefetch=$p $(tail -1 $O/bench_p$p.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["value"],2), round(d["ms_per_step"],2))')"
done
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -T -d $O/prof -o bench --output-format csv -- python3 $ROOT/bench.py --steps 2 --warmup 2 --no-cpu-baseline > $O/prof.log 2>&1 || { echo "prof failed"; tail -5 $O/prof.log; exit 1; }
cd $ROOT && python3 tools/prof_summary.py $O/prof/bench_kernel_trace.csv --steps 2 --accum 4 --out $O/timed.csv --top 12 > $O/timed.txt || { echo "summary failed"; exit 2; }
head -6 $O/timed.txt
echo all-ok
