#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT
for o in 2 4 8; do
  SKP_BGEMM_OCC=$o timeout -k 10 60 python -u tools/kbench.py --only gemm16,gemm32 --iters 20 > gpurun_out/occ_$o.txt 2>&1 || { cat gpurun_out/occ_$o.txt; exit 2; }
  echo "occ $o: $(grep -E '_(fwd|dq|dk) ' gpurun_out/occ_$o.txt | awk '{printf "%s %s  ", $1, $2}')"
done
