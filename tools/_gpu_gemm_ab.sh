#!/bin/bash
# bgemm A/B: parity (bgemm + capture logits + token-opt step), then kbench gemm16/32 vs build/var_old
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu -k "bgemm or capture_logits or token_opt" -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/gemm_ab_tests.log 2>&1 || { tail -30 gpurun_out/gemm_ab_tests.log; exit 1; }
tail -1 gpurun_out/gemm_ab_tests.log
for i in 1 2; do
  echo "new: $(timeout -k 10 60 python -u tools/kbench.py --only gemm16,gemm32 --iters 20 2>&1 | grep -E '_(fwd|dq|dk) ' | awk '{printf "%s %s  ", $1, $2}')"
  echo "old: $(SKP_LIB=build/var_old/libskp.so timeout -k 10 60 python -u tools/kbench.py --only gemm16,gemm32 --iters 20 2>&1 | grep -E '_(fwd|dq|dk) ' | awk '{printf "%s %s  ", $1, $2}')"
done
