#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
ROOT=$GRAFT_REPO_ROOT
O=$ROOT/gpurun_out/r03p
mkdir -p $O
cd /tmp
HOST_ORDER=after timeout -k 10 400 rocprofv3 --hip-runtime-trace --kernel-trace -d $O/hip -o h --output-format csv -- python3 $ROOT/tools/host_time.py --steps 4 > $O/hip.log 2>&1 || { echo "hip trace failed"; tail -20 $O/hip.log; exit 1; }
grep "step\|host issued" $O/hip.log
cd $ROOT
python3 - <<'PY'
import csv, glob
rows = list(csv.DictReader(open(glob.glob("gpurun_out/r03p/hip/*hip_api_trace.csv")[0])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
t_end = int(rows[-1]["End_Timestamp"])
win = [r for r in rows if int(r["Start_Timestamp"]) > t_end - 600_000_000]
long = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]), int(r["Start_Timestamp"]), r["Function"]) for r in win]
long = [x for x in long if x[0] > 500_000]
print("API calls > 0.5 ms in the last 600 ms:", len(long))
t0 = int(win[0]["Start_Timestamp"])
for d, s, f in long[:60]:
    print(f"  t={(s - t0) / 1e6:8.2f} ms  {d / 1e6:7.2f} ms  {f}")
PY
echo all-ok
