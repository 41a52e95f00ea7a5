#!/bin/bash
# SDXL bench (configs[4], 1024², N=500) on the final round-3 tree (Winograd-GEMM form included)
set -o pipefail
export TMPDIR=/tmp
ROOT=$GRAFT_REPO_ROOT
O=$ROOT/gpurun_out/r03bb
mkdir -p $O
cd $ROOT
timeout -k 10 800 python -u bench.py --model sdxl --steps 3 --warmup 2 --no-cpu-baseline > $O/bench_sdxl.log 2>&1 || { echo "sdxl bench failed rc=$?"; grep -v amdgpu $O/bench_sdxl.log | tail -30; exit 1; }
tail -1 $O/bench_sdxl.log | cut -c1-300
