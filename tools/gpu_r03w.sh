#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
ROOT=$GRAFT_REPO_ROOT
O=$ROOT/gpurun_out/r03w
mkdir -p $O
cd $ROOT
timeout -k 10 300 python -u tools/gemm_eff.py --rows 60 --isolated > $O/gemm_eff.log 2>&1 || { echo "gemm_eff failed rc=$?"; grep -v amdgpu $O/gemm_eff.log | tail -20 | cut -c1-300; exit 1; }
grep -v amdgpu $O/gemm_eff.log | head -64 | cut -c1-200
