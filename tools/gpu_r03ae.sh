#!/bin/bash
# fused capture forward: non-temporal map/stats stores (default build) vs plain stores
# (build/variants/libskp_plain.so): tests, kernel time, FETCH_SIZE, bench
set -o pipefail
export TMPDIR=/tmp
ROOT=$GRAFT_REPO_ROOT
O=$ROOT/gpurun_out/r03ae
mkdir -p $O
cd $ROOT
PLAIN=$ROOT/build/variants/libskp_plain.so
DEF=$ROOT/stablekeypoints_amd/libskp.so
timeout -k 10 300 python -u -m pytest -x -q -p no:cacheprovider --timeout 120 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_sel_bwd.py -m gpu -k "capture_maps or sel" > $O/tests.log 2>&1 || { echo "tests failed"; grep -v amdgpu $O/tests.log | tail -20; exit 4; }
tail -1 $O/tests.log
for v in def plain def plain; do
  if [ $v = plain ]; then L=$PLAIN; else L=$DEF; fi
  SKP_LIB=$L timeout -k 10 200 python -u tools/kbench.py --only maps8 --iters 20 > $O/kb_$v.log 2>&1 || { echo "kbench failed"; tail -5 $O/kb_$v.log; exit 2; }
  echo "$v $(grep maps8 $O/kb_$v.log)"
done
cd /tmp
for v in def plain; do
  if [ $v = plain ]; then L=$PLAIN; else L=$DEF; fi
  SKP_LIB=$L timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $O/pmc_f$v -o c --output-format csv -- python3 $ROOT/tools/kbench.py --only maps8 --iters 3 > $O/pmc_f$v.log 2>&1 || { echo "pmc failed"; exit 3; }
  python3 -c "
import csv,statistics
v=[float(r['Counter_Value']) for r in csv.DictReader(open('$O/pmc_f$v/c_counter_collection.csv')) if 'capture_maps' in r['Kernel_Name']]
print('$v FETCH MB', statistics.median(v)*2*1024/1e6)"
done
cd $ROOT
for v in def plain; do
  if [ $v = plain ]; then L=$PLAIN; else L=$DEF; fi
  SKP_LIB=$L timeout -k 10 400 python -u bench.py --steps 8 --warmup 3 --no-cpu-baseline > $O/bench_$v.log 2>&1 || { echo "bench failed"; tail -5 $O/bench_$v.log; exit 5; }
  tail -1 $O/bench_$v.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$v', round(d['value'],3), 'fwd', round(d['roofline']['avg_launch_ms'],4), 'frac', round(d['roofline']['frac'],4))"
done
