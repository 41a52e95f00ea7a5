#!/bin/bash
# fused backward with float4 transpose / vertical adjoint: parity, A/B timing, per-kernel trace
set -o pipefail
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/bwdvec
mkdir -p $O
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu -k "capture_maps or batched or token_opt" -p no:cacheprovider --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for i in 1 2; do
timeout -k 10 120 python -u tools/kbench.py --only mapsbwd8 --iters 20 > $O/k1.txt 2>&1 || { cat $O/k1.txt; exit 2; }
SKP_LIB=build/var_oldbwd/libskp.so timeout -k 10 120 python -u tools/kbench.py --only mapsbwd8 --iters 20 > $O/k2.txt 2>&1 || { cat $O/k2.txt; exit 3; }
echo "new: $(grep maps $O/k1.txt)   old: $(grep maps $O/k2.txt)"
done
cd /tmp && timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/prof -o k --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/kbench.py --only mapsbwd8 --iters 10 > $O/prof.log 2>&1 || { tail -3 $O/prof.log; exit 4; }
grep -E "transpose|cols|row_kernel" $O/prof/k_kernel_stats.csv | cut -d, -f1-8
