#!/bin/bash
# Round-3: sparse backward (reworked) + BSHD attention: tests, kernel timings, bench, untruncated
# elementwise names of one bench step.  Each GPU step under its own limit; stop at the first failure.
set -o pipefail
export TMPDIR=/tmp
ROOT=$GRAFT_REPO_ROOT
O=$ROOT/gpurun_out/r03c
mkdir -p $O
cd $ROOT
PT="python -u -m pytest -x -v -p no:cacheprovider --timeout 120 --timeout-method thread"
timeout -k 10 400 $PT tests/test_gpu_sel_bwd.py tests/test_gpu_attn_bshd.py -m gpu > $O/tests.log 2>&1 || { echo "tests failed rc=$?"; tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 200 python -u tools/kbench.py --only mapssel8,mapssel8_dense --iters 10 > $O/kbench.log 2>&1 || { echo "kbench failed"; tail -20 $O/kbench.log; exit 2; }
cat $O/kbench.log
timeout -k 10 600 python -u bench.py --no-cpu-baseline > $O/bench.log 2>&1 || { echo "bench failed rc=$?"; tail -30 $O/bench.log; exit 3; }
tail -1 $O/bench.log | cut -c1-400
SKP_ATTN_BSHD=0 timeout -k 10 600 python -u bench.py --no-cpu-baseline > $O/bench_nobshd.log 2>&1 || { echo "bench nobshd failed rc=$?"; tail -30 $O/bench_nobshd.log; exit 4; }
tail -1 $O/bench_nobshd.log | cut -c1-200
cd /tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/kprof -o k --output-format csv -- python3 $ROOT/tools/kbench.py --only mapssel8 --iters 5 > $O/kprof.log 2>&1 || { echo "kprof failed"; exit 5; }
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/ntprof -o b --output-format csv -- python3 $ROOT/bench.py --steps 1 --warmup 1 --no-cpu-baseline > $O/ntprof.log 2>&1 || { echo "ntprof failed"; exit 6; }
cd $ROOT && python3 tools/elementwise_names.py $O/ntprof/b_kernel_trace.csv > $O/elementwise_names.txt && head -30 $O/elementwise_names.txt | cut -c1-250
python3 - <<'PY'
import csv
for r in csv.DictReader(open("gpurun_out/r03c/kprof/k_kernel_stats.csv")):
    if "sel_" in r["Name"]:
        print(f'{r["Name"][:60]:60s} calls {r["Calls"]:>4s} avg {float(r["AverageNs"])/1e3:9.1f} us')
PY
echo all-ok
