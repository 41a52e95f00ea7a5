#!/bin/bash
# Round profiles: bench with CPU baseline (JSON line), SDXL bench, rocprofv3 kernel-trace stats of
# the bench and its timed-region summary.  Each step under its own limit; stops at the first failure.
set -o pipefail
R=${1:-r01}
export TMPDIR=/tmp
ROOT=$GRAFT_REPO_ROOT
mkdir -p $ROOT/gpurun_out/refresh
O=$ROOT/gpurun_out/refresh
cd $ROOT
timeout -k 10 400 python -u bench.py > $O/bench.log 2>&1 || { echo "bench failed"; tail -20 $O/bench.log; exit 1; }
tail -1 $O/bench.log > $O/bench.json
timeout -k 10 400 python -u bench.py --model sdxl --no-cpu-baseline > $O/bench_sdxl.log 2>&1 || { echo "sdxl bench failed"; tail -20 $O/bench_sdxl.log; exit 2; }
tail -1 $O/bench_sdxl.log > $O/bench_sdxl.json
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -T -d $O/prof -o bench --output-format csv -- python $ROOT/bench.py --steps 2 --warmup 2 --no-cpu-baseline > $O/prof.log 2>&1 || { echo "prof failed"; tail -20 $O/prof.log; exit 3; }
cd $ROOT
python tools/prof_summary.py $O/prof/bench_kernel_trace.csv --micro 8 --out $O/timed_summary.csv --top 40 > $O/timed_summary.txt
cut -c1-200 $O/bench.json; cut -c1-120 $O/bench_sdxl.json; head -3 $O/timed_summary.txt
echo refresh-ok
