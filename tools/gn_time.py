"""Dev tool: time the fused GroupNorm(+SiLU) forward and backward (skp_groupnorm_fwd/bwd) at UNet/VAE shapes.

usage: python tools/gn_time.py [--shapes B,C,HW;...]  (SKP_LIB selects an A/B build)
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from stablekeypoints_amd import ops

ap = argparse.ArgumentParser()
ap.add_argument("--shapes", default="8,128,512;8,256,256;8,512,128;8,320,64;8,640,32;8,1280,16")
ap.add_argument("--iters", type=int, default=10)
a = ap.parse_args()


def timed(f):
    f()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(a.iters):
        f()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / a.iters * 1e3


for s in a.shapes.split(";"):
    B, C, HW = map(int, s.split(","))
    x = torch.randn(B, C, HW, HW, device="cuda:0", requires_grad=True)
    g = torch.rand(C, device="cuda:0") + 0.5
    b = torch.randn(C, device="cuda:0")
    t_f = timed(lambda: ops.group_norm_act(x.detach(), g, b, 32, 1e-5, True))
    y = ops.group_norm_act(x, g, b, 32, 1e-5, True)
    dy = torch.randn_like(y)
    t_b = timed(lambda: torch.autograd.grad(y, x, dy, retain_graph=True))
    gb = x.numel() * 4 / 1e9
    print(f"{B}x{C}x{HW}^2: fwd {t_f:8.1f} us ({3 * gb / (t_f * 1e-6) / 1e3:5.2f} TB/s of 3 passes)  "
          f"bwd {t_b:8.1f} us ({5 * gb / (t_b * 1e-6) / 1e3:5.2f} TB/s of 5 passes)", flush=True)
