#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
ROOT=$GRAFT_REPO_ROOT
O=$ROOT/gpurun_out/r03b
mkdir -p $O
cd $ROOT
timeout -k 10 300 python -u -m pytest -x -v -p no:cacheprovider --timeout 120 --timeout-method thread tests/test_gpu_sel_bwd.py -m gpu > $O/sel_tests.log 2>&1 || { echo "sel tests failed rc=$?"; tail -40 $O/sel_tests.log; exit 1; }
tail -1 $O/sel_tests.log
timeout -k 10 200 python -u tools/kbench.py --only mapssel8,mapssel8_dense --iters 10 > $O/kbench.log 2>&1 || { echo "kbench failed"; tail -20 $O/kbench.log; exit 2; }
cat $O/kbench.log
cd /tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/kprof -o k --output-format csv -- python3 $ROOT/tools/kbench.py --only mapssel8 --iters 5 > $O/kprof.log 2>&1 || { echo "kprof failed"; exit 3; }
grep -E "sel_" $O/kprof/k_kernel_stats.csv | cut -d, -f1-8
timeout -s KILL 90 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_INSTS_VALU GRBM_GUI_ACTIVE --kernel-trace -d $O/pmc_valu -o c --output-format csv -- python3 $ROOT/tools/kbench.py --only mapssel8 --iters 2 > $O/pmc_valu.log 2>&1 || { echo "pmc valu failed"; exit 4; }
cd $ROOT && python3 - <<'PY'
import csv, collections
per = collections.defaultdict(dict)
for r in csv.DictReader(open("gpurun_out/r03b/pmc_valu/c_counter_collection.csv")):
    per[(r["Dispatch_Id"], r["Kernel_Name"][:48])][r["Counter_Name"]] = float(r["Counter_Value"])
for (d, k), v in per.items():
    if "sel_" in k:
        print(k, int(v["SQ_INSTS_VALU"]), f'busy {4*v["SQ_ACTIVE_INST_VALU"]/(1024*v["GRBM_GUI_ACTIVE"]/8):.3f}')
PY
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/ntprof -o b --output-format csv -- python3 $ROOT/bench.py --steps 1 --warmup 1 --no-cpu-baseline > $O/ntprof.log 2>&1 || { echo "ntprof failed"; exit 5; }
cd $ROOT && python3 - <<'PY'
import csv, collections
rows = list(csv.DictReader(open("gpurun_out/r03b/ntprof/b_kernel_trace.csv")))
agg = collections.defaultdict(lambda: [0, 0.0])
for r in rows:
    n = r["Kernel_Name"]
    if "elementwise_kernel" in n or "transpose" in n:
        d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        import re
        key = (re.sub(r"\s+", " ", n)[:700], r["Grid_Size_X"])
        agg[key][0] += 1; agg[key][1] += d
with open("gpurun_out/r03b/elementwise_names.txt", "w") as f:
    for (n, g), (c, t) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:60]:
        f.write(f"{t/1e3:8.3f} ms {c:4d} grid {g:>10s}  {n}\n")
print("names written")
PY
