#!/bin/bash
# HIP-graph pass: the graph-vs-eager test, the token-opt / refapi / distributed tests, then a bench
# A/B (graph replay vs eager launches, alternating) and smoke.  Each step under its own limit.
set -o pipefail
export TMPDIR=/tmp
ROOT=$GRAFT_REPO_ROOT
O=$ROOT/gpurun_out/r03t
mkdir -p $O
cd $ROOT
PT="python -u -m pytest -x -v -p no:cacheprovider --timeout 120 --timeout-method thread"
timeout -k 10 300 python -u tools/graph_try.py --tiny > $O/gtiny.log 2>&1 || { echo "graph_try tiny failed rc=$?"; grep -v amdgpu $O/gtiny.log | grep -v "^  File" | tail -20 | cut -c1-300; exit 1; }
grep -v amdgpu $O/gtiny.log | tail -4
timeout -k 10 400 $PT tests/test_gpu_graph.py tests/test_gpu_refapi.py -m gpu > $O/tests.log 2>&1 || { echo "tests failed rc=$?"; grep -v amdgpu $O/tests.log | tail -40 | cut -c1-300; exit 1; }
tail -1 $O/tests.log
for g in 1 0 1 0; do
  timeout -k 10 400 python -u bench.py --graph $g --steps 8 --warmup 3 --no-cpu-baseline > $O/bench_g$g.log 2>&1 || { echo "bench graph=$g failed rc=$?"; grep -v amdgpu $O/bench_g$g.log | tail -30 | cut -c1-300; exit 2; }
  tail -1 $O/bench_g$g.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('graph', $g, d['value'], d['ms_per_step'], d['roofline']['achieved'], d['last_loss'])"
done
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $O/smoke.log; exit 3; }
tail -2 $O/smoke.log
echo all-ok
