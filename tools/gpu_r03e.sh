#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
ROOT=$GRAFT_REPO_ROOT
O=$ROOT/gpurun_out/r03e
mkdir -p $O
cd $ROOT
timeout -k 10 300 python -u tools/attn_bshd_time.py > $O/attn.log 2>&1 || { echo "attn failed"; tail -20 $O/attn.log; exit 1; }
grep -v amdgpu.ids $O/attn.log
cd /tmp
ATTN_ONLY=self timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/aprof -o a --output-format csv -- python3 $ROOT/tools/attn_bshd_time.py --iters 5 > $O/aprof.log 2>&1 || { echo "aprof failed"; exit 2; }
cd $ROOT && python3 - <<'PY'
import csv
for r in csv.DictReader(open("gpurun_out/r03e/aprof/a_kernel_stats.csv")):
    print(f'{r["Name"][:90]:90s} calls {r["Calls"]:>4s} avg {float(r["AverageNs"])/1e3:9.1f} us tot {float(r["TotalDurationNs"])/1e3:9.1f}')
PY
cd /tmp
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-trace -d $O/pmc_lds -o c --output-format csv -- python3 $ROOT/tools/kbench.py --only maps8,mapssel8 --iters 2 > $O/pmc_lds.log 2>&1 || { echo "pmc lds failed"; exit 4; }
cd $ROOT && python3 - <<'PY'
import csv, collections
per = collections.defaultdict(dict)
for r in csv.DictReader(open("gpurun_out/r03e/pmc_lds/c_counter_collection.csv")):
    per[(r["Dispatch_Id"], r["Kernel_Name"][:48])][r["Counter_Name"]] = float(r["Counter_Value"])
seen = set()
for (d, k), v in per.items():
    if ("sel_dense" in k or "capture_maps" in k) and k not in seen:
        seen.add(k)
        g = v["GRBM_GUI_ACTIVE"] / 8
        print(k, {a: int(b) for a, b in v.items()}, f'lds_active/CU-cycle {v["SQ_LDS_IDX_ACTIVE"] / 256 / g:.3f}')
PY
echo all-ok
