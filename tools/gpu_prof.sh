#!/bin/bash
# Profiles for the round: kernel-trace stats of the bench (timed region summarised by
# tools/prof_summary.py --steps), PMC HBM counters in separate passes for skp_aggregate via the
# kernel micro-benchmark, and the micro-benchmark's kernel stats.  Output under gpurun_out/.
set -o pipefail
R=${1:-r01}
mkdir -p gpurun_out
export TMPDIR=/tmp
ROOT=$GRAFT_REPO_ROOT
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -T -d $ROOT/gpurun_out/prof_$R -o bench --output-format csv -- python $ROOT/bench.py --steps 2 --warmup 1 --no-cpu-baseline > $ROOT/gpurun_out/prof_$R.log 2>&1 || exit 1
timeout -k 10 200 rocprofv3 --pmc FETCH_SIZE --kernel-trace -T -d $ROOT/gpurun_out/pmc_fetch_$R -o agg --output-format csv -- python $ROOT/tools/kbench.py --only agg --iters 5 > /dev/null 2>&1 || exit 2
timeout -k 10 200 rocprofv3 --pmc WRITE_SIZE --kernel-trace -T -d $ROOT/gpurun_out/pmc_write_$R -o agg --output-format csv -- python $ROOT/tools/kbench.py --only agg --iters 5 > /dev/null 2>&1 || exit 3
timeout -k 10 200 rocprofv3 --kernel-trace --stats -T -d $ROOT/gpurun_out/kprof_$R -o kb --output-format csv -- python $ROOT/tools/kbench.py > $ROOT/gpurun_out/kbench_$R.log 2>&1 || exit 4
cd $ROOT && python tools/prof_summary.py gpurun_out/prof_$R/bench_kernel_trace.csv --steps 2 --accum 4 --out gpurun_out/prof_${R}_timed.csv > gpurun_out/prof_${R}_timed.txt
echo done
