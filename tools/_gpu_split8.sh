set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
python -c "
from stablekeypoints_amd import ops
for C in (1280, 2560): print(C, ops._wino_plan(8, C, 1280, 8, 8))
"
for s in 0 4 5 8 10 16 20; do
  SKP_WINO_NSPLIT=$s timeout -k 10 120 python -u tools/conv8_probe.py > gpurun_out/s8.log 2>&1 || { tail -5 gpurun_out/s8.log; exit 1; }
  echo "nsplit=$s: $(grep 'C=' gpurun_out/s8.log | cut -c1-40 | tr '\n' ' ')"
done
