#!/bin/bash
# copy-site attribution of one pass on the current tree; bench A/B: VAE prefetch on a side stream (1)
# vs the VAE on the main stream (0), alternating
set -o pipefail
export TMPDIR=/tmp
ROOT=$GRAFT_REPO_ROOT
O=$ROOT/gpurun_out/r03ar
mkdir -p $O
cd $ROOT
timeout -k 10 300 python -u tools/copy_sites.py --rows 80 > $O/copy_sites.log 2>&1 || { echo "copy_sites failed rc=$?"; grep -v amdgpu $O/copy_sites.log | tail -20 | cut -c1-300; exit 1; }
grep -v amdgpu $O/copy_sites.log | head -45 | cut -c1-250
for v in 0 1 0 1; do
  timeout -k 10 400 python -u bench.py --steps 8 --warmup 3 --no-cpu-baseline --prefetch $v > $O/bench_$v.log 2>&1 || { echo "bench failed"; tail -5 $O/bench_$v.log; exit 4; }
  tail -1 $O/bench_$v.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('prefetch=$v', round(d['value'],3), round(d['ms_per_step'],2))"
done
