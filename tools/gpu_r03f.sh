#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
ROOT=$GRAFT_REPO_ROOT
O=$ROOT/gpurun_out/r03f
mkdir -p $O
cd $ROOT
timeout -k 10 400 python -u -m pytest -x -q -p no:cacheprovider --timeout 120 --timeout-method thread tests/test_gpu_sel_bwd.py tests/test_gpu_attn_bshd.py -m gpu > $O/tests.log 2>&1 || { echo "tests failed rc=$?"; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 200 python -u tools/kbench.py --only mapssel8,maps8 --iters 10 > $O/kbench.log 2>&1 || { echo "kbench failed"; exit 2; }
grep -v amdgpu $O/kbench.log
for v in 1 0 1 0; do
  SKP_ATTN_BSHD=$v timeout -k 10 400 python -u bench.py --no-cpu-baseline --steps 4 > $O/bench_$v.log 2>&1 || { echo "bench $v failed"; tail -20 $O/bench_$v.log; exit 3; }
  echo "BSHD=$v $(tail -1 $O/bench_$v.log | cut -c1-160)"
done
cd /tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/kprof -o k --output-format csv -- python3 $ROOT/tools/kbench.py --only mapssel8 --iters 5 > $O/kprof.log 2>&1 || { echo "kprof failed"; exit 4; }
cd $ROOT && python3 - <<'PY'
import csv
for r in csv.DictReader(open("gpurun_out/r03f/kprof/k_kernel_stats.csv")):
    if "sel_" in r["Name"]:
        print(f'{r["Name"][:60]:60s} calls {r["Calls"]:>4s} avg {float(r["AverageNs"])/1e3:9.1f} us')
PY
echo all-ok
