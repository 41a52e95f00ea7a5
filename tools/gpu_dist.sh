#!/bin/bash
# Rehearse bench.py's world-size-2 path on a one-GPU box: both ranks on cuda:0, gloo instead of RCCL
set -o pipefail
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/${RUN_TAG:-dist}
mkdir -p $O
cd $GRAFT_REPO_ROOT
SKP_BENCH_ONE_DEVICE=1 SKP_BENCH_DIST_BACKEND=gloo timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29531 bench.py --gpus 2 --steps 2 --warmup 1 > $O/bench2.log 2>&1 || { echo "rc=$?"; tail -30 $O/bench2.log; exit 1; }
grep '"metric"' $O/bench2.log
