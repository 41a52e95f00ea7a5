#!/bin/bash
# rocprofv3 kernel trace + stats of tools/kbench.py --only $1; prints the stats table
set -o pipefail
export TMPDIR=/tmp
ROOT=$GRAFT_REPO_ROOT
OUT=$ROOT/gpurun_out/prof_$1
cd /tmp && timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $OUT -o k --output-format csv -- python3 $ROOT/tools/kbench.py --only $1 --iters ${2:-5} > $OUT.log 2>&1 || { echo "prof failed"; tail -5 $OUT.log; exit 1; }
f=$(find $OUT -name "*kernel_stats.csv" | head -1)
python3 - "$f" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
for r in rows[:12]:
    print(f'{float(r["TotalDurationNs"])/1e3:10.1f} us  n={r["Calls"]:>4}  avg={float(r["AverageNs"])/1e3:8.1f} us  {r["Name"][:100]}')
PY
