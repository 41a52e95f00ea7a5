#!/bin/bash
# rocprofv3 kernel-trace stats of kbench entries (KB) under environment settings (dev tool):
#   KB=kl4 bash tools/gpu_kb_prof_env.sh "SKP_X=0" "SKP_X=1"
set -o pipefail
export TMPDIR=/tmp
ROOT=$GRAFT_REPO_ROOT
O=$ROOT/gpurun_out/${RUN_TAG:-kbprof}
mkdir -p $O
cd /tmp
i=0
for e in "$@"; do
  i=$((i+1))
  export $e
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/p$i -o kb --output-format csv -- python3 $ROOT/tools/kbench.py --only $KB --iters ${KB_ITERS:-20} > $O/p$i.log 2>&1 || { echo "prof ($e) failed"; tail -5 $O/p$i.log; exit 8; }
  unset ${e%%=*}
  echo "== $e"
  python3 - "$O/p$i" <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True)[0]
rows = sorted(csv.DictReader(open(f)), key=lambda r: -float(r["TotalDurationNs"]))
for r in rows[:12]:
    print(f'{r["Name"][:80]:80s} {int(r["Calls"]):6d} {float(r["AverageNs"]) / 1e3:10.1f} us')
PY
done
