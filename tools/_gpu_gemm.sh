#!/bin/bash
# bgemm parity + timing at the capture shapes (default tiles, then the 64×64-only A/B form)
set -o pipefail
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/gemm
mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu -k "bgemm or logits or capture_maps or token_opt" -p no:cacheprovider --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 120 python -u tools/kbench.py --only gemm16,gemm32 --iters 20 > $O/kbench.txt 2>&1 || { cat $O/kbench.txt; exit 2; }
echo "default: $(grep -E '_(fwd|dq|dk) ' $O/kbench.txt | awk '{printf "%s %s  ", $1, $2}')"
SKP_BGEMM_TILE=64 timeout -k 10 120 python -u tools/kbench.py --only gemm16,gemm32 --iters 20 > $O/kbench64.txt 2>&1 || { cat $O/kbench64.txt; exit 3; }
echo "tile64:  $(grep -E '_(fwd|dq|dk) ' $O/kbench64.txt | awk '{printf "%s %s  ", $1, $2}')"
SKP_BGEMM_WAVES=4 timeout -k 10 120 python -u tools/kbench.py --only gemm16,gemm32 --iters 20 > $O/kbench4w.txt 2>&1 || { cat $O/kbench4w.txt; exit 4; }
echo "4waves:  $(grep -E '_(fwd|dq|dk) ' $O/kbench4w.txt | awk '{printf "%s %s  ", $1, $2}')"
