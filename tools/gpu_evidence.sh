#!/bin/bash
# Round-3 evidence refresh on the committed tree: smoke, default bench (with cpu_baseline), the
# eval-stage benches, kernel timings, a timed-region kernel trace, the whole GPU suite and the PMC
# passes (capture forward per layer size, sparse backward) — each step under its own limit.  A GPU
# fault / abort / timeout ends the script; test assertion failures (pytest rc 1) are recorded and
# the measurements continue.
set -o pipefail
export TMPDIR=/tmp
ROOT=$GRAFT_REPO_ROOT
O=$ROOT/gpurun_out/${RUN_TAG:-r03x}
mkdir -p $O
cd $ROOT
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $O/smoke.log; exit 3; }
grep -v amdgpu $O/smoke.log | tail -3
timeout -k 10 600 python -u bench.py > $O/bench.log 2>&1 || { echo "bench failed rc=$?"; tail -30 $O/bench.log; exit 4; }
tail -1 $O/bench.log | cut -c1-300
for t in 100 500; do
  timeout -k 10 300 python -u bench.py --stage find_indices --tokens $t --steps 3 --warmup 1 > $O/bench_find_$t.log 2>&1 || { echo "find_indices $t failed rc=$?"; tail -30 $O/bench_find_$t.log; exit 5; }
  tail -1 $O/bench_find_$t.log | cut -c1-200
done
timeout -k 10 300 python -u bench.py --stage tta --steps 2 --warmup 1 --stage-images 4 > $O/bench_tta.log 2>&1 || { echo "tta failed rc=$?"; tail -30 $O/bench_tta.log; exit 6; }
tail -1 $O/bench_tta.log | cut -c1-200
timeout -k 10 200 python -u tools/kbench.py --only maps8,maps8_s16,maps8_s32,mapsbwd8,mapssel8,mapssel8_dense --iters 10 > $O/kbench.log 2>&1 || { echo "kbench failed"; tail -20 $O/kbench.log; exit 7; }
grep -v amdgpu $O/kbench.log
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof -o bench --output-format csv -- python3 $ROOT/bench.py --steps 2 --warmup 2 --no-cpu-baseline > $O/prof.log 2>&1 || { echo "prof failed"; tail -5 $O/prof.log; exit 9; }
cd $ROOT && python3 tools/prof_summary.py $O/prof/bench_kernel_trace.csv --steps 2 --accum 4 --out $O/timed_summary.csv --top 45 > $O/timed_summary.txt || { echo "summary failed"; exit 10; }
head -8 $O/timed_summary.txt | cut -c1-150
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?
tail -3 $O/gpu_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest aborted rc=$rc"; exit 11; fi
cd /tmp
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $c --kernel-trace -d $O/pmc_$c -o c --output-format csv -- python3 $ROOT/tools/kbench.py --only maps8,maps8_s16,maps8_s32,mapssel8 --iters 3 > $O/pmc_$c.log 2>&1 || { echo "pmc $c failed"; exit 12; }
done
timeout -s KILL 120 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_INSTS_VALU GRBM_GUI_ACTIVE --kernel-trace -d $O/pmc_valu -o c --output-format csv -- python3 $ROOT/tools/kbench.py --only maps8,mapssel8 --iters 3 > $O/pmc_valu.log 2>&1 || { echo "pmc valu failed"; exit 13; }
find $O -name "*counter_collection.csv"
echo "all-ok (full suite rc=$rc)"
