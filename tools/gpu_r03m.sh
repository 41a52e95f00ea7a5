#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
ROOT=$GRAFT_REPO_ROOT
O=$ROOT/gpurun_out/r03m
mkdir -p $O
cd /tmp
HOST_ORDER=before timeout -k 10 400 rocprofv3 --hip-runtime-trace --stats -d $O/hip -o h --output-format csv -- python3 $ROOT/tools/host_time.py --steps 4 > $O/hip.log 2>&1 || { echo "hip trace failed"; tail -20 $O/hip.log; exit 1; }
grep -v amdgpu $O/hip.log | tail -5
cd $ROOT
ls $O/hip
python3 - <<'PY'
import csv, glob
f = glob.glob("gpurun_out/r03m/hip/*hip_api_stats.csv")
if f:
    rows = list(csv.DictReader(open(f[0])))
    rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
    for r in rows[:25]:
        print(f'{r["Name"][:40]:40s} calls {r["Calls"]:>7s} total {float(r["TotalDurationNs"])/1e6:9.2f} ms avg {float(r["AverageNs"])/1e3:9.1f} us max {float(r["MaxNs"])/1e3:9.1f} us')
PY
echo all-ok
