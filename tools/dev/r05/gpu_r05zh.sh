#!/bin/bash
# r05zh: streamed KL kernel timing probes (1: no window pass, 2: no window pass, no reductions)
# and a torch read of the same maps (dev script; probe keys are wrong by construction)
set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/r05zh; mkdir -p $O
KB=kl4 RUN_TAG=r05zh_prof bash tools/gpu_kb_prof_env.sh SKP_KL_PROBE=0 SKP_KL_PROBE=1 SKP_KL_PROBE=2 || exit 1
timeout -k 10 120 python -u - <<'PY'
import torch
m = torch.rand(4, 500, 128, 128, device="cuda") ** 8
for name, fn in (("sum", lambda: m.sum()), ("amax", lambda: m.amax(dim=(2, 3)))):
    fn(); torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(20): fn()
    b.record(); torch.cuda.synchronize()
    t = a.elapsed_time(b) / 20
    print(f"torch {name} over the kl4 maps: {t * 1e3:.1f} us = {m.numel() * 4 / t / 1e9:.2f} TB/s")
PY
echo r05zh-ok
