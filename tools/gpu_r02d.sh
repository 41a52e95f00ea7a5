#!/bin/bash
# Round-2 (session c, final) evidence: GPU tests, smoke, default bench, timed-region kernel trace, PMC
# passes (maps traffic + VALU, backward VALU, bgemm MFMA-busy) — each step under its own limit,
# stopping at the first failure.
set -o pipefail
export TMPDIR=/tmp
ROOT=$GRAFT_REPO_ROOT
O=$ROOT/gpurun_out/r02d
mkdir -p $O
cd $ROOT
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo "pytest failed rc=$?"; tail -40 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $O/smoke.log; exit 2; }
timeout -k 10 600 python -u bench.py > $O/bench.log 2>&1 || { echo "bench failed rc=$?"; tail -30 $O/bench.log; exit 3; }
tail -1 $O/bench.log
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -T -d $O/prof -o bench --output-format csv -- python3 $ROOT/bench.py --steps 2 --warmup 2 --no-cpu-baseline > $O/prof.log 2>&1 || { echo "prof failed"; tail -5 $O/prof.log; exit 4; }
cd $ROOT && python3 tools/prof_summary.py $O/prof/bench_kernel_trace.csv --steps 2 --accum 4 --out $O/timed_summary.csv --top 45 > $O/timed_summary.txt || { echo "summary failed"; exit 5; }
head -3 $O/timed_summary.txt
cd /tmp
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 90 rocprofv3 --pmc $c --kernel-trace -d $O/pmc_$c -o c --output-format csv -- python3 $ROOT/tools/kbench.py --only maps8 --iters 3 > $O/pmc_$c.log 2>&1 || { echo "pmc $c failed"; exit 6; }
done
timeout -s KILL 90 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_VALU_TRANS_F32 GRBM_GUI_ACTIVE --kernel-trace -d $O/pmc_valu -o c --output-format csv -- python3 $ROOT/tools/kbench.py --only maps8,mapsbwd8 --iters 3 > $O/pmc_valu.log 2>&1 || { echo "pmc valu failed"; exit 7; }
timeout -s KILL 90 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-trace -d $O/pmc_mfma -o c --output-format csv -- python3 $ROOT/tools/kbench.py --only gemm16,gemm32 --iters 3 > $O/pmc_mfma.log 2>&1 || { echo "pmc mfma failed"; exit 8; }
cd $ROOT
python3 tools/pmc_summary.py $O/pmc_mfma --match bgemm > $O/pmc_mfma_bgemm.txt; grep -E "bgemm|MFMA busy" $O/pmc_mfma_bgemm.txt | head -20
timeout -s KILL 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-trace -d $O/pmc_wino -o c --output-format csv -- python3 $ROOT/bench.py --steps 1 --warmup 1 --no-cpu-baseline > $O/pmc_wino.log 2>&1 || { echo "pmc wino failed"; exit 9; }
cd $ROOT
python3 tools/pmc_summary.py $O/pmc_wino --match wino > $O/pmc_mfma_wino.txt; grep -E "wino|MFMA busy|VALU busy" $O/pmc_mfma_wino.txt | head -20
find $O -name "*counter_collection.csv" | head
echo all-ok
