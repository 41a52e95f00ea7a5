#!/bin/bash
set -o pipefail
export TMPDIR=/tmp
ROOT=$GRAFT_REPO_ROOT
O=$ROOT/gpurun_out/r03ab
mkdir -p $O
cd $ROOT
timeout -k 10 900 python -u bench.py --model sdxl --steps 3 --warmup 2 > $O/bench_sdxl.log 2>&1 || { echo "sdxl bench failed rc=$?"; grep -v amdgpu $O/bench_sdxl.log | tail -30; exit 1; }
tail -1 $O/bench_sdxl.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['roofline'].get('avg_launch_ms'), {k: v.get('avg_ms') for k, v in d['kernels'].items()})"
