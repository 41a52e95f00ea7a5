"""A/B of the resnet shortcut 1×1 convolutions at the bench's batch (8): ops.conv1x1 (one batched
GEMM on NCHW) vs F.conv2d (MIOpen), forward + input gradient (dev tool)."""
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from stablekeypoints_amd import ops  # noqa: E402


def timed(fn, iters=20):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / iters * 1e3


# UNet shortcuts on the bench's path (down 320→640 @32², 640→1280 @16², up 2560→1280 @8²/16²,
# 1920→1280 @16², 1920→640 @32², 1280→640 @32², 960→640 @32²) and the VAE's (128→256 @256², 256→512 @128²)
for C, K, H, grad in ((320, 640, 32, True), (640, 1280, 16, True), (2560, 1280, 8, True), (2560, 1280, 16, True),
                      (1920, 1280, 16, True), (1920, 640, 32, True), (1280, 640, 32, True), (960, 640, 32, True),
                      (128, 256, 256, False), (256, 512, 128, False)):
    x = torch.randn(8, C, H, H, device="cuda", requires_grad=grad)
    w = torch.randn(K, C, 1, 1, device="cuda") / C ** 0.5
    dy = torch.randn(8, K, H, H, device="cuda")

    def run(f):
        if grad:
            y = f()
            torch.autograd.backward(y, dy)
        else:
            with torch.no_grad():
                f()
    t_g = timed(lambda: run(lambda: ops.conv1x1(x, w)))
    t_m = timed(lambda: run(lambda: F.conv2d(x, w)))
    print(f"{C:5d}->{K:5d} @{H:3d}² {'fwd+bwd' if grad else 'fwd'}: GEMM {t_g:8.1f} us  MIOpen {t_m:8.1f} us", flush=True)
