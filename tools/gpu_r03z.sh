#!/bin/bash
# merged small sparse-backward kernels + VAE prefetch after the capture backward: tests, kernel
# timings, bench A/B (prefetch placement), each step under its own limit
set -o pipefail
export TMPDIR=/tmp
ROOT=$GRAFT_REPO_ROOT
O=$ROOT/gpurun_out/r03z
mkdir -p $O
cd $ROOT
PT="python -u -m pytest -x -q -p no:cacheprovider --timeout 120 --timeout-method thread"
timeout -k 10 400 $PT tests/test_gpu_sel_bwd.py tests/test_gpu_graph.py tests/test_gpu_parity.py -m gpu -k "sel or graph or micro_steps or prefetch or token_opt or step" > $O/tests.log 2>&1 || { echo "tests failed rc=$?"; grep -v amdgpu $O/tests.log | grep -v "^  File" | tail -30 | cut -c1-300; exit 1; }
tail -1 $O/tests.log
timeout -k 10 200 python -u tools/kbench.py --only mapssel8,mapssel8_dense --iters 10 > $O/kbench.log 2>&1 || { echo "kbench failed"; tail -20 $O/kbench.log; exit 2; }
grep -v amdgpu $O/kbench.log
cd /tmp
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/kprof -o k --output-format csv -- python3 $ROOT/tools/kbench.py --only mapssel8 --iters 5 > $O/kprof.log 2>&1 || { echo "kprof failed"; exit 3; }
grep -E "sel_" $O/kprof/k_kernel_stats.csv | cut -d, -f1-4 | cut -c1-160
cd $ROOT
for p in capture_bwd bwd capture_bwd bwd; do
  timeout -k 10 400 python -u bench.py --prefetch-at $p --steps 8 --warmup 3 --no-cpu-baseline > $O/bench_$p.log 2>&1 || { echo "bench $p failed rc=$?"; tail -20 $O/bench_$p.log; exit 4; }
  tail -1 $O/bench_$p.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); k=d['kernels'].get('skp_capture_maps_bwd_sel',{}); print('$p', round(d['value'],3), round(d['ms_per_step'],2), 'fwd', round(d['roofline']['avg_launch_ms'],3), 'selbwd', round(k.get('avg_ms',0),3))"
done
