set -o pipefail
cd $GRAFT_REPO_ROOT
echo default; timeout -k 10 200 python -u tools/conv_probe.py --vae --batch 8 2>&1 | grep -E " s2|total" || exit 1
echo no-igemm; MIOPEN_DEBUG_CONV_IMPLICIT_GEMM=0 timeout -k 10 200 python -u tools/conv_probe.py --vae --batch 8 2>&1 | grep -E " s2|total" || exit 2
echo no-igemm-bench; MIOPEN_DEBUG_CONV_IMPLICIT_GEMM=0 timeout -k 10 300 python -u tools/conv_probe.py --vae --batch 8 --benchmark 2>&1 | grep -E " s2|total" || exit 3
echo channels-last; timeout -k 10 200 python -u tools/conv_probe.py --vae --batch 8 --channels-last 2>&1 | grep -E " s2|total" || exit 4
