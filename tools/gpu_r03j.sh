#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
ROOT=$GRAFT_REPO_ROOT
O=$ROOT/gpurun_out/r03j
mkdir -p $O
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -T -d $O/prof -o bench --output-format csv -- python3 $ROOT/bench.py --steps 2 --warmup 2 --no-cpu-baseline > $O/prof.log 2>&1 || { echo "prof failed"; tail -5 $O/prof.log; exit 1; }
cd $ROOT && python3 tools/prof_summary.py $O/prof/bench_kernel_trace.csv --steps 2 --accum 4 --out $O/timed.csv --top 40 > $O/timed.txt || { echo "summary failed"; exit 2; }
head -44 $O/timed.txt
echo all-ok
