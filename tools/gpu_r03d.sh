#!/bin/bash
# A/B of the BSHD attention: micro timings, then timed-region kernel summaries of the bench with and
# without it (same box).
set -o pipefail
export TMPDIR=/tmp
ROOT=$GRAFT_REPO_ROOT
O=$ROOT/gpurun_out/r03d
mkdir -p $O
cd $ROOT
timeout -k 10 300 python -u -m pytest -x -q -p no:cacheprovider --timeout 120 --timeout-method thread tests/test_gpu_sel_bwd.py -m gpu > $O/sel_tests.log 2>&1 || { echo "sel tests failed rc=$?"; tail -30 $O/sel_tests.log; exit 1; }
tail -1 $O/sel_tests.log
cd /tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/kprof -o k --output-format csv -- python3 $ROOT/tools/kbench.py --only mapssel8 --iters 5 > $O/kprof.log 2>&1 || { echo "kprof failed"; exit 1; }
timeout -s KILL 90 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAVES GRBM_GUI_ACTIVE --kernel-trace -d $O/pmc_valu -o c --output-format csv -- python3 $ROOT/tools/kbench.py --only mapssel8 --iters 2 > $O/pmc_valu.log 2>&1 || { echo "pmc valu failed"; exit 1; }
cd $ROOT && python3 - <<'PY'
import csv, collections
for r in csv.DictReader(open("gpurun_out/r03d/kprof/k_kernel_stats.csv")):
    if "sel_" in r["Name"]:
        print(f'{r["Name"][:60]:60s} calls {r["Calls"]:>4s} avg {float(r["AverageNs"])/1e3:9.1f} us')
per = collections.defaultdict(dict)
for r in csv.DictReader(open("gpurun_out/r03d/pmc_valu/c_counter_collection.csv")):
    per[(r["Dispatch_Id"], r["Kernel_Name"][:48])][r["Counter_Name"]] = float(r["Counter_Value"])
seen = set()
for (d, k), v in per.items():
    if "sel_" in k and k not in seen:
        seen.add(k)
        print(k, int(v["SQ_INSTS_VALU"]), f'busy {4*v["SQ_ACTIVE_INST_VALU"]/(1024*v["GRBM_GUI_ACTIVE"]/8):.3f}')
PY
timeout -k 10 300 python -u tools/attn_bshd_time.py > $O/attn.log 2>&1 || { echo "attn failed"; tail -20 $O/attn.log; exit 1; }
cat $O/attn.log | grep -v amdgpu.ids
cd /tmp
for v in 1 0; do
  SKP_ATTN_BSHD=$v timeout -k 10 400 rocprofv3 --kernel-trace --stats -T -d $O/prof$v -o bench --output-format csv -- python3 $ROOT/bench.py --steps 2 --warmup 2 --no-cpu-baseline > $O/prof$v.log 2>&1 || { echo "prof $v failed"; tail -5 $O/prof$v.log; exit 2; }
  cd $ROOT && python3 tools/prof_summary.py $O/prof$v/bench_kernel_trace.csv --steps 2 --accum 4 --out $O/timed$v.csv --top 30 > $O/timed$v.txt || { echo "summary failed"; exit 3; }
  head -14 $O/timed$v.txt
  cd /tmp
done
echo all-ok
cd /tmp
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-trace -d $ROOT/gpurun_out/r03d/pmc_lds -o c --output-format csv -- python3 $ROOT/tools/kbench.py --only maps8,mapssel8 --iters 2 > $ROOT/gpurun_out/r03d/pmc_lds.log 2>&1 || { echo "pmc lds failed"; exit 4; }
cd $ROOT && python3 - <<'PY'
import csv, collections
per = collections.defaultdict(dict)
for r in csv.DictReader(open("gpurun_out/r03d/pmc_lds/c_counter_collection.csv")):
    per[(r["Dispatch_Id"], r["Kernel_Name"][:48])][r["Counter_Name"]] = float(r["Counter_Value"])
seen = set()
for (d, k), v in per.items():
    if ("sel_dense" in k or "capture_maps" in k) and k not in seen:
        seen.add(k)
        g = v["GRBM_GUI_ACTIVE"] / 8
        print(k, {a: int(b) for a, b in v.items()}, f'lds_active/CU-cycle {v["SQ_LDS_IDX_ACTIVE"] / 256 / g:.3f}')
PY
