"""Attribute device time of one token-opt optimiser step (4 images + warps, batch-8 pass,
forward + backward) to torch ops and their callers (dev tool).

For every aten op with device time: its input shapes, and its caller — the nearest repo
frame of its Python stack (forward) or the autograd node that ran it (backward).  Prints
the top rows by device time, grouped by (op, caller, shapes).

    python tools/op_attrib.py [--rows 80] [--match copy,clone,contiguous,add,mul,cat]
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from torch.profiler import ProfilerActivity, profile

from stablekeypoints_amd.datasets import SyntheticDataset
from stablekeypoints_amd.optimize import TokenOptimizer
from stablekeypoints_amd.optimize_token import load_ldm

ap = argparse.ArgumentParser()
ap.add_argument("--rows", type=int, default=80)
ap.add_argument("--match", default="")
args = ap.parse_args()

dev = torch.device("cuda:0")
ldm, ctls, _ = load_ldm(dev, "random", feature_upsample_res=128)
torch.manual_seed(0)
ctx = torch.randn(1, 500, 768).to(dev)
opt = TokenOptimizer(ldm, ctls, ctx, accum=4, device=dev)
imgs = [SyntheticDataset(n=4, size=512)[i]["img"][None].to(dev) for i in range(4)]
for _ in range(2):
    opt.micro_steps(imgs)
torch.cuda.synchronize()
with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], record_shapes=True, with_stack=True) as prof:
    opt.micro_steps(imgs)
    torch.cuda.synchronize()


def dev_time(e):
    return getattr(e, "self_device_time_total", 0) or getattr(e, "self_cuda_time_total", 0)


def caller(e):
    p = e
    while p is not None:
        if p.name.startswith("autograd::engine::evaluate_function"):
            return "bwd:" + p.name.split(":", 4)[-1].strip()
        st = [f for f in (p.stack or []) if "stablekeypoints_amd" in f or "tools/" in f]
        if st:
            f = st[0]
            return "fwd:" + f.split("stablekeypoints_amd/")[-1][:90]
        p = p.cpu_parent
    return "?"


# stack-grouped table of the copy-like ops (the Python call sites of every strided copy / memcpy)
ka = prof.key_averages(group_by_stack_n=6)
rows_s = [k for k in ka if any(n in k.key for n in ("copy_", "clone", "contiguous", "cat", "_to_copy", "fill_", "add"))]
rows_s.sort(key=lambda k: -(getattr(k, "self_device_time_total", 0) or 0))
print("--- copy-like ops by Python stack (self device time)")
for k in rows_s[:40]:
    t = getattr(k, "self_device_time_total", 0) or 0
    if t <= 0:
        continue
    st = [f for f in (k.stack or []) if "torch/" not in f][:4]
    print(f"{t / 1e3:8.3f} ms {k.count:4d} {k.key:24s} {str(k.input_shapes)[:70]:70s} | " + " <- ".join(st))
match = [m for m in args.match.split(",") if m]
rows = {}
total = 0.0
for e in prof.events():
    t = dev_time(e)
    if t <= 0 or not e.name.startswith("aten::"):
        continue
    total += t
    if match and not any(m in e.name for m in match):
        continue
    key = (e.name, caller(e), str(e.input_shapes)[:110])
    r = rows.setdefault(key, [0.0, 0])
    r[0] += t
    r[1] += 1
print(f"aten device time in one optimiser step: {total / 1e3:.2f} ms")
for (name, who, sh), (t, n) in sorted(rows.items(), key=lambda kv: -kv[1][0])[:args.rows]:
    print(f"{t / 1e3:8.3f} ms {n:4d} {name:28s} {who:60s} {sh}")
by_op = {}
for (name, who, sh), (t, n) in rows.items():
    a = by_op.setdefault((name, who), [0.0, 0])
    a[0] += t
    a[1] += n
print("--- by (op, caller)")
for (name, who), (t, n) in sorted(by_op.items(), key=lambda kv: -kv[1][0])[:60]:
    print(f"{t / 1e3:8.3f} ms {n:4d} {name:28s} {who}")
