#!/bin/bash
# A round's evidence refresh on the committed tree, part PART (default "bench"):
#   bench: smoke, the default bench (with cpu_baseline), STAGE_RUNS (default 3) runs each of the
#          eval-stage benches, rocprofv3 kernel traces of the token-opt bench and both stages,
#          timed-region summaries; DIST=1: bench.py --gpus 2 on one GPU (gloo); SDXL=1: configs[4]
#   suite: the whole -m gpu suite (-s: the parity prints), then the PMC passes (tools/gpu_pmc.sh)
# Each step runs under its own limit; a GPU fault / abort / timeout ends the script.
set -o pipefail
export TMPDIR=/tmp
ROOT=$GRAFT_REPO_ROOT
TAG=${RUN_TAG:-r04x}
O=$ROOT/gpurun_out/$TAG
mkdir -p $O
cd $ROOT
if [ "${PART:-bench}" = "bench" ]; then
  timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $O/smoke.log; exit 3; }
  grep -v amdgpu $O/smoke.log | tail -3
  timeout -k 10 600 python -u bench.py > $O/bench.log 2>&1 || { echo "bench failed rc=$?"; tail -30 $O/bench.log; exit 4; }
  tail -1 $O/bench.log | cut -c1-300
  for i in $(seq 1 ${STAGE_RUNS:-3}); do
    timeout -k 10 300 python -u bench.py --stage find_indices --tokens 100 --steps 3 --warmup 1 > $O/bench_find_100_$i.log 2>&1 || { echo "find_indices failed rc=$?"; tail -30 $O/bench_find_100_$i.log; exit 5; }
    tail -1 $O/bench_find_100_$i.log | cut -c1-120
    timeout -k 10 300 python -u bench.py --stage tta --steps 2 --warmup 1 --stage-images 4 > $O/bench_tta_$i.log 2>&1 || { echo "tta failed rc=$?"; tail -30 $O/bench_tta_$i.log; exit 6; }
    tail -1 $O/bench_tta_$i.log | cut -c1-120
  done
  timeout -k 10 300 python -u bench.py --stage find_indices --tokens 500 --steps 3 --warmup 1 > $O/bench_find_500.log 2>&1 || { echo "find_indices 500 failed"; exit 5; }
  tail -1 $O/bench_find_500.log | cut -c1-120
  cd /tmp
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/prof -o bench --output-format csv -- python3 $ROOT/bench.py --steps 2 --warmup 2 --no-cpu-baseline > $O/prof.log 2>&1 || { echo "prof failed"; tail -5 $O/prof.log; exit 9; }
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_find -o find --output-format csv -- python3 $ROOT/bench.py --stage find_indices --tokens 100 --steps 3 --warmup 1 > $O/prof_find.log 2>&1 || { echo "prof find failed"; tail -5 $O/prof_find.log; exit 9; }
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_tta -o tta --output-format csv -- python3 $ROOT/bench.py --stage tta --steps 2 --warmup 1 --stage-images 4 > $O/prof_tta.log 2>&1 || { echo "prof tta failed"; tail -5 $O/prof_tta.log; exit 9; }
  cd $ROOT
  python3 tools/prof_summary.py $O/prof/bench_kernel_trace.csv --steps 2 --accum 4 --out $O/timed_summary.csv --top 45 > $O/timed_summary.txt || { echo "summary failed"; exit 10; }
  head -4 $O/timed_summary.txt | cut -c1-150
  for st in find tta; do
    ms=$(python3 -c "import json; d=json.loads([l for l in open('$O/prof_$st.log').read().splitlines() if l.startswith('{\"metric\"')][-1]); print(d['ms_per_step'] * d['steps'])")
    n=$(python3 -c "import json; d=json.loads([l for l in open('$O/prof_$st.log').read().splitlines() if l.startswith('{\"metric\"')][-1]); print(d['config']['images_per_step'] * d['steps'])")
    python3 tools/prof_summary.py $O/prof_$st/${st}_kernel_trace.csv --tail-ms $ms --images $n --out $O/timed_summary_$st.csv --top 30 > $O/timed_summary_$st.txt || { echo "summary $st failed"; exit 10; }
    head -3 $O/timed_summary_$st.txt | cut -c1-150
  done
  if [ -n "$DIST" ]; then   # the world-2 path through bench.py --gpus 2, both ranks on cuda:0 over gloo
    SKP_BENCH_ONE_DEVICE=1 SKP_BENCH_DIST_BACKEND=gloo timeout -k 10 600 python -u bench.py --gpus 2 --steps 3 --warmup 1 --no-cpu-baseline > $O/bench_gpus2.log 2>&1 || { echo "bench --gpus 2 failed rc=$?"; tail -20 $O/bench_gpus2.log; exit 14; }
    grep '^{' $O/bench_gpus2.log | tail -1 | cut -c1-200
  fi
  if [ -n "$SDXL" ]; then
    timeout -k 10 600 python -u bench.py --model sdxl --steps 3 --warmup 1 > $O/bench_sdxl.log 2>&1 || { echo "sdxl failed rc=$?"; tail -20 $O/bench_sdxl.log; exit 15; }
    grep '^{' $O/bench_sdxl.log | tail -1 | cut -c1-200
  fi
  echo "bench-ok"
else
  timeout -k 10 1000 python -u -m pytest tests -x -q -s -m gpu -p no:cacheprovider --timeout 150 --timeout-method thread > $O/gpu_tests.log 2>&1
  rc=$?
  tail -3 $O/gpu_tests.log
  if [ $rc -ne 0 ]; then echo "pytest rc=$rc"; exit 11; fi
  RUN_TAG=$TAG/pmc bash tools/gpu_pmc.sh || exit 12
  echo "suite-ok"
fi
