#!/bin/bash
# Timing probes of the fused capture forward (no vertical-pass loads / staging only) + baselines
set -o pipefail
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/diag
mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 120 python -u tools/kbench.py --only maps8,mapsbwd8,gemm16,gemm32 --iters 20 > $O/base.txt 2>&1 || { cat $O/base.txt; exit 1; }
cat $O/base.txt
for v in d1 d2; do
  SKP_LIB=build/var_$v/libskp.so timeout -k 10 120 python -u tools/kbench.py --only maps8 --iters 20 > $O/$v.txt 2>&1 || { cat $O/$v.txt; exit 2; }
  echo "$v: $(cat $O/$v.txt)"
done
