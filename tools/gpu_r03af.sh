#!/bin/bash
# bench A/B, alternating: non-temporal capture stores (default build) vs plain (variant build)
set -o pipefail
export TMPDIR=/tmp
ROOT=$GRAFT_REPO_ROOT
O=$ROOT/gpurun_out/r03af
mkdir -p $O
cd $ROOT
for v in plain def plain def; do
  if [ $v = plain ]; then L=$ROOT/build/variants/libskp_plain.so; else L=$ROOT/stablekeypoints_amd/libskp.so; fi
  SKP_LIB=$L timeout -k 10 400 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline > $O/bench_$v.log 2>&1 || { echo "bench failed"; tail -5 $O/bench_$v.log; exit 5; }
  tail -1 $O/bench_$v.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$v', round(d['value'],3), 'fwd', round(d['roofline']['avg_launch_ms'],4), 'sel', round(d['kernels']['skp_capture_maps_bwd_sel']['avg_ms'],4))"
done
