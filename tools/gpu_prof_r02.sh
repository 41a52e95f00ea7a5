#!/bin/bash
# Round-2 evidence: default bench, timed-region kernel trace, PMC traffic + VALU for the fused
# capture kernel (kbench at the bench shape), MFMA-busy of the convolutions over the whole bench.
set -o pipefail
export TMPDIR=/tmp
ROOT=$GRAFT_REPO_ROOT
O=$ROOT/gpurun_out/r02
mkdir -p $O
cd $ROOT
timeout -k 10 600 python -u bench.py > $O/bench.log 2>&1 || { echo "bench failed rc=$?"; tail -20 $O/bench.log; exit 1; }
tail -1 $O/bench.log
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -T -d $O/prof -o bench --output-format csv -- python3 $ROOT/bench.py --steps 2 --warmup 2 --no-cpu-baseline > $O/prof.log 2>&1 || { echo "prof failed"; tail -5 $O/prof.log; exit 2; }
cd $ROOT && python3 tools/prof_summary.py $O/prof/bench_kernel_trace.csv --steps 2 --accum 4 --out $O/timed_summary.csv --top 40 > $O/timed_summary.txt || { echo "summary failed"; exit 3; }
head -25 $O/timed_summary.txt
cd /tmp
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 90 rocprofv3 --pmc $c --kernel-trace -d $O/pmc_$c -o c --output-format csv -- python3 $ROOT/tools/kbench.py --only maps8 --iters 3 > $O/pmc_$c.log 2>&1 || { echo "pmc $c failed"; exit 4; }
done
timeout -s KILL 90 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_VALU_TRANS_F32 GRBM_GUI_ACTIVE --kernel-trace -d $O/pmc_valu -o c --output-format csv -- python3 $ROOT/tools/kbench.py --only maps8,mapsbwd8 --iters 3 > $O/pmc_valu.log 2>&1 || { echo "pmc valu failed"; exit 5; }
timeout -s KILL 300 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-trace -d $O/pmc_mfma -o c --output-format csv -- python3 $ROOT/bench.py --steps 1 --warmup 1 --no-cpu-baseline > $O/pmc_mfma.log 2>&1 || { echo "pmc mfma failed"; exit 6; }
cd $ROOT
python3 tools/pmc_summary.py $O/pmc_mfma --match wino > $O/pmc_mfma_wino.txt; head -30 $O/pmc_mfma_wino.txt
echo all-ok
