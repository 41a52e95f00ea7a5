#!/bin/bash
# persistent capture-forward grid: bit-exact test, kernel time A/B, FETCH_SIZE A/B
set -o pipefail
export TMPDIR=/tmp
ROOT=$GRAFT_REPO_ROOT
O=$ROOT/gpurun_out/r03ad
mkdir -p $O
cd $ROOT
timeout -k 10 300 python -u -m pytest -x -q -p no:cacheprovider --timeout 120 --timeout-method thread tests/test_gpu_parity.py -m gpu -k "capture_maps" > $O/tests.log 2>&1 || { echo "tests failed rc=$?"; grep -v amdgpu $O/tests.log | grep -v "^  File" | tail -30 | cut -c1-300; exit 1; }
tail -1 $O/tests.log
for p in 1 0 1 0; do
  SKP_MAPS_PERSIST=$p timeout -k 10 200 python -u tools/kbench.py --only maps8 --iters 20 > $O/kb_$p.log 2>&1 || { echo "kbench failed"; exit 2; }
  echo "persist=$p $(grep maps8 $O/kb_$p.log)"
done
cd /tmp
for p in 1 0; do
  SKP_MAPS_PERSIST=$p timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $O/pmc_f$p -o c --output-format csv -- python3 $ROOT/tools/kbench.py --only maps8 --iters 3 > $O/pmc_f$p.log 2>&1 || { echo "pmc failed"; exit 3; }
  python3 -c "
import csv,statistics
v=[float(r['Counter_Value']) for r in csv.DictReader(open('$O/pmc_f$p/c_counter_collection.csv')) if 'capture_maps' in r['Kernel_Name']]
print('persist=$p FETCH_SIZE median KB', statistics.median(v), '-> MB x2', statistics.median(v)*2*1024/1e6)"
done
