#!/bin/bash
# bench A/B: the pass on a high-priority stream vs the default stream (alternating)
set -o pipefail
export TMPDIR=/tmp
ROOT=$GRAFT_REPO_ROOT
O=$ROOT/gpurun_out/r03ai
mkdir -p $O
cd $ROOT
for v in 1 0 1 0; do
  timeout -k 10 400 python -u bench.py --main-priority $v --steps 10 --warmup 3 --no-cpu-baseline > $O/bench_$v.log 2>&1 || { echo "bench failed"; tail -8 $O/bench_$v.log; exit 3; }
  tail -1 $O/bench_$v.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('prio=$v', round(d['value'],3), round(d['ms_per_step'],2), 'fwd', round(d['roofline']['avg_launch_ms'],3), 'sel', round(d['kernels']['skp_capture_maps_bwd_sel']['avg_ms'],3))"
done
