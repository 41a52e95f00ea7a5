"""Timing of the VAE's stride-2 downsampling convolutions at the bench batch (8 = 4 images + 4
warps): the stride-2 Winograd path (ops.conv3x3_s2) vs F.pad + MIOpen conv2d(stride 2) (dev tool)."""
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from stablekeypoints_amd import ops  # noqa: E402


def timed(fn, iters=10):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / iters * 1e3


with torch.no_grad():
    for C, H in ((128, 512), (256, 256), (512, 128)):
        x = torch.randn(8, C, H, H, device="cuda")
        w = torch.randn(C, C, 3, 3, device="cuda") * 0.02
        b = torch.randn(C, device="cuda")
        t_w = timed(lambda: ops.conv3x3_s2(x, w, b))
        t_m = timed(lambda: F.conv2d(F.pad(x, (0, 1, 0, 1)), w, b, stride=2))
        print(f"{C:4d} ch {H}²: stride-2 Winograd {t_w:8.1f} us   pad + MIOpen {t_m:8.1f} us", flush=True)
