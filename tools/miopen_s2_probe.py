"""The VAE's stride-2 convolutions at 256² and 128² (batch 8) through MIOpen under the current
environment (run once per MIOpen setting: solver switches are read per process), with and without
torch.backends.cudnn.benchmark (exhaustive find) — F.pad + conv2d(stride 2) (dev tool)."""
import os
import sys

import torch
import torch.nn.functional as F

bench = "--find" in sys.argv
torch.backends.cudnn.benchmark = bench


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


tag = os.environ.get("PROBE_TAG", "default") + (" +find" if bench else "")
with torch.no_grad():
    for C, H in ((256, 256), (512, 128)):
        x = torch.randn(8, C, H, H, device="cuda")
        w = torch.randn(C, C, 3, 3, device="cuda") * 0.02
        b = torch.randn(C, device="cuda")
        xp = F.pad(x, (0, 1, 0, 1))
        t_conv = timed(lambda: F.conv2d(xp, w, b, stride=2))
        t_all = timed(lambda: F.conv2d(F.pad(x, (0, 1, 0, 1)), w, b, stride=2))
        ref = F.conv2d(xp.double(), w.double(), b.double(), stride=2)
        err = (F.conv2d(xp, w, b, stride=2).double() - ref).abs().max().item() / ref.abs().max().item()
        print(f"{tag:40s} {C:4d} ch {H}²: conv {t_conv:8.1f} us  pad+conv {t_all:8.1f} us  rel err {err:.1e}", flush=True)
