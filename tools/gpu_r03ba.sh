#!/bin/bash
# find_best_indices stage A/B: Winograd-GEMM form (SKP_WINO_GEMM_MAX_HW=1024, default) vs the fused
# kernels (0) — r03az measured 67.5 it/s at N=100 against r03aq's 77.7 before the GEMM form
set -o pipefail
export TMPDIR=/tmp
ROOT=$GRAFT_REPO_ROOT
O=$ROOT/gpurun_out/r03ba
mkdir -p $O
cd $ROOT
for v in 1024 0 1024 0; do
  for t in 100 500; do
    SKP_WINO_GEMM_MAX_HW=$v timeout -k 10 300 python -u bench.py --stage find_indices --tokens $t --steps 6 --warmup 2 > $O/find_${v}_$t.log 2>&1 || { echo "find_indices failed"; tail -20 $O/find_${v}_$t.log; exit 2; }
    tail -1 $O/find_${v}_$t.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('MAX_HW=$v N=$t', round(d['value'],2), round(d['ms_per_step'],2))"
  done
done
