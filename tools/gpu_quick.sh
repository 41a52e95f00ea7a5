#!/bin/bash
# Quick GPU check: the named test files (TESTS, default the whole -m gpu suite) and optional
# kbench entries (KB); each step under its own limit, stops at the first GPU fault/abort/timeout.
set -o pipefail
export TMPDIR=/tmp
ROOT=$GRAFT_REPO_ROOT
O=$ROOT/gpurun_out/${RUN_TAG:-quick}
mkdir -p $O
cd $ROOT
if [ -n "$KB" ]; then
  timeout -k 10 200 python -u tools/kbench.py --only $KB --iters ${KB_ITERS:-20} > $O/kbench.log 2>&1 || { echo "kbench failed"; tail -20 $O/kbench.log; exit 7; }
  grep -v amdgpu $O/kbench.log
fi
if [ -n "$PROF" ]; then   # rocprofv3 kernel-trace stats of kbench --only $PROF
  cd /tmp
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o kb --output-format csv -- python3 $ROOT/tools/kbench.py --only $PROF --iters ${KB_ITERS:-20} > $O/prof.log 2>&1 || { echo "prof failed"; tail -20 $O/prof.log; exit 8; }
  cd $ROOT
  python3 - "$O" <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/prof/**/*kernel_stats.csv", recursive=True)[0]
rows = sorted(csv.DictReader(open(f)), key=lambda r: -float(r["TotalDurationNs"]))
for r in rows[:25]:
    print(f'{r["Name"][:90]:90s} {int(r["Calls"]):6d} {float(r["AverageNs"]) / 1e3:10.1f} us')
PY
fi
if [ "${TESTS:-all}" != "none" ]; then
  T=${TESTS:-tests}
  timeout -k 10 ${TEST_LIMIT:-900} python -u -m pytest $T -x -q -m gpu -p no:cacheprovider --timeout 120 --timeout-method thread ${PYTEST_ARGS:-} > $O/gpu_tests.log 2>&1
  rc=$?
  tail -15 $O/gpu_tests.log
  if [ $rc -ne 0 ]; then echo "pytest rc=$rc"; exit 11; fi
fi
if [ -n "$BENCH" ]; then
  timeout -k 10 600 python -u bench.py $BENCH > $O/bench.log 2>&1 || { echo "bench failed rc=$?"; tail -30 $O/bench.log; exit 4; }
  tail -1 $O/bench.log | cut -c1-400
fi
echo all-ok
