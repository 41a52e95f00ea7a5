"""Per-shape efficiency of the step's library GEMMs (hipBLASLt via aten mm / addmm / bmm / baddbmm /
linear) in one token-opt pass (4 images + warps, batch-8 forward + backward, plus the next pass's
VAE prefetch): device time, FLOPs and TF/s per (op, shapes), largest total first (dev tool).

    python tools/gemm_eff.py [--rows 50]
"""
import argparse
import collections
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from torch.profiler import ProfilerActivity, profile

from stablekeypoints_amd.datasets import SyntheticDataset
from stablekeypoints_amd.optimize import TokenOptimizer
from stablekeypoints_amd.optimize_token import load_ldm

ap = argparse.ArgumentParser()
ap.add_argument("--rows", type=int, default=50)
ap.add_argument("--isolated", action="store_true", help="no VAE prefetch running beside the pass")
OPT = ap.parse_args()

dev = torch.device("cuda:0")
ldm, ctls, _ = load_ldm(dev, "random", feature_upsample_res=128)
torch.manual_seed(0)
ctx = torch.randn(1, 500, 768).to(dev)
opt = TokenOptimizer(ldm, ctls, ctx, accum=4, device=dev)
data = SyntheticDataset(n=8, size=512)
imgs = [data[i]["img"][None].to(dev) for i in range(8)]
opt.micro_steps(imgs[:4])
opt.optimizer_step()
opt.prefetch(imgs[4:])
torch.cuda.synchronize()
with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], record_shapes=True) as prof:
    opt.micro_steps(imgs[4:], prefetch=[] if OPT.isolated else [imgs[:4]])
    torch.cuda.synchronize()


def flops(name, shapes):
    try:
        if name in ("aten::mm",):
            (m, k), (_, n) = shapes[0], shapes[1]
            return 2 * m * k * n
        if name == "aten::addmm":
            (m, k), (_, n) = shapes[1], shapes[2]
            return 2 * m * k * n
        if name == "aten::bmm":
            (b, m, k), (_, _, n) = shapes[0], shapes[1]
            return 2 * b * m * k * n
        if name == "aten::baddbmm":
            (b, m, k), (_, _, n) = shapes[1], shapes[2]
            return 2 * b * m * k * n
    except (ValueError, TypeError, IndexError):
        return 0
    return 0


rows = collections.defaultdict(lambda: [0, 0.0, 0])
for e in prof.events():
    if e.name not in ("aten::mm", "aten::addmm", "aten::bmm", "aten::baddbmm"):
        continue
    t = getattr(e, "device_time_total", 0) or getattr(e, "cuda_time_total", 0)
    if t <= 0:
        continue
    key = (e.name, str(e.input_shapes)[:90])
    r = rows[key]
    r[0] += 1
    r[1] += t
    r[2] += flops(e.name, e.input_shapes)
tot_t = sum(r[1] for r in rows.values())
tot_f = sum(r[2] for r in rows.values())
print(f"library GEMMs in one pass: {tot_t / 1e3:.2f} ms, {tot_f / 1e12:.2f} TFLOP, "
      f"{tot_f / (tot_t * 1e-6) / 1e12:.1f} TF/s (f32 MFMA dense peak 157.3)")
for (name, sh), (n, t, f) in sorted(rows.items(), key=lambda kv: -kv[1][1])[:OPT.rows]:
    tf = f / (t * 1e-6) / 1e12 if t else 0
    print(f"{t / 1e3:8.3f} ms {n:3d} {tf:6.1f} TF/s  {name:14s} {sh}")
