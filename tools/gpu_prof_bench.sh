#!/bin/bash
# Timed-region kernel profile of bench.py under rocprofv3 (kernel trace only).
set -o pipefail
R=${1:-r01}
mkdir -p gpurun_out
export TMPDIR=/tmp
ROOT=$GRAFT_REPO_ROOT
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -T -d $ROOT/gpurun_out/prof_$R -o bench --output-format csv -- python $ROOT/bench.py --steps 2 --warmup 2 --no-cpu-baseline > $ROOT/gpurun_out/prof_$R.log 2>&1 || exit 1
cd $ROOT && python tools/prof_summary.py gpurun_out/prof_$R/bench_kernel_trace.csv --micro 8 --out gpurun_out/prof_$R/timed_summary.csv --top 40
