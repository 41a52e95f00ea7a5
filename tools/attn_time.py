"""Dev tool: time the fused attention kernels at the UNet's 64²-token self-attention shape
(BH = 64, S = L = 4096, d = 40): forward-only (skp_attn_fwd) and flash forward + backward.

usage: python tools/attn_time.py  (SKP_LIB selects an A/B build)
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from stablekeypoints_amd import ops

dev = "cuda:0"
BH, S, L, d = 64, 4096, 4096, 40
g = torch.Generator(device=dev).manual_seed(0)
q = torch.randn(BH, S, d, device=dev, generator=g, requires_grad=True)
k = torch.randn(BH, L, d, device=dev, generator=g, requires_grad=True)
v = torch.randn(BH, L, d, device=dev, generator=g, requires_grad=True)


def timed(fn, iters=10):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / iters


with torch.no_grad():
    t_nog = timed(lambda: ops.attention_nograd(q, k, v, d ** -0.5))
out = ops.math_attention(q, k, v, d ** -0.5)
dout = torch.randn_like(out)
t_fwd = timed(lambda: ops.math_attention(q, k, v, d ** -0.5))
t_bwd = timed(lambda: torch.autograd.grad(out, (q, k, v), dout, retain_graph=True))
fl = 4 * BH * S * L * d
print(f"attn 64^2 d=40: nograd fwd {t_nog * 1e3:7.1f} us ({fl / t_nog / 1e9:5.1f} TF/s)  "
      f"flash fwd {t_fwd * 1e3:7.1f} us  bwd {t_bwd * 1e3:7.1f} us", flush=True)
