"""Dev probe: skp LayerNorm vs ATen at the UNet transformer shapes (batch 8), forward and backward."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from stablekeypoints_amd import ops

ops.LN_MIN_ROWS = 1


def t(f, it=100):
    for _ in range(3):
        f()
    torch.cuda.synchronize()
    a, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(it):
        f()
    e.record(); torch.cuda.synchronize()
    return a.elapsed_time(e) / it * 1e3


for shape in ((8, 4096, 320), (8, 1024, 640), (8, 256, 1280)):
    x = torch.randn(*shape, device="cuda:0"); w = torch.randn(shape[-1], device="cuda:0"); b = torch.randn_like(w)
    C = shape[-1]
    y = torch.empty_like(x); st = torch.empty(x.numel() // C, 2, device="cuda:0")
    from stablekeypoints_amd._lib import call, ptr, stream
    k = lambda: call("skp_layernorm_fwd", ptr(x), ptr(w), ptr(b), x.numel() // C, C, 1e-5, ptr(y), ptr(st), stream("cuda:0"))
    dx = torch.empty_like(x)
    kb = lambda: call("skp_layernorm_bwd", ptr(x), ptr(x), ptr(w), ptr(st), x.numel() // C, C, ptr(dx), stream("cuda:0"))
    t1, t2 = t(k), t(kb)
    t0 = t(lambda: torch.nn.functional.layer_norm(x, (C,), w, b, 1e-5))
    print(shape, f"skp fwd {t1:.1f} us ({2 * x.numel() * 4 / t1 / 1e3:.0f} GB/s) bwd {t2:.1f} us  torch fwd {t0:.1f} us", flush=True)
