"""torch.profiler op-level attribution of one token-opt micro-iteration (dev tool)."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from torch.profiler import profile, ProfilerActivity
from stablekeypoints_amd.optimize import TokenOptimizer
from stablekeypoints_amd.optimize_token import load_ldm
from stablekeypoints_amd.datasets import SyntheticDataset

dev = torch.device("cuda:0")
ldm, ctls, _ = load_ldm(dev, "random", feature_upsample_res=128)
torch.manual_seed(0)
ctx = torch.randn(1, 500, 768).to(dev)
opt = TokenOptimizer(ldm, ctls, ctx, accum=4, device=dev)
imgs = [SyntheticDataset(n=4, size=512)[i]["img"][None].to(dev) for i in range(4)]
for _ in range(2):
    opt.micro_steps(imgs)
torch.cuda.synchronize()
import sys as _s
shapes = "--shapes" in _s.argv
with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], record_shapes=shapes) as prof:
    opt.micro_steps(imgs)   # one optimiser step's 4 images in one batch-8 pass
    torch.cuda.synchronize()
if shapes:
    rows = []
    for e in prof.key_averages(group_by_input_shape=True):
        t = getattr(e, "self_device_time_total", 0) or getattr(e, "self_cuda_time_total", 0)
        if e.key.startswith("aten::") and t > 0:
            rows.append((t, e.key, e.count, str(e.input_shapes)[:150]))
    rows.sort(reverse=True)
    for t, k, n, sh in rows[:int(os.environ.get("ROWS", "120"))]:
        print(f"{t / 1e3:8.3f} ms {n:5d} {k:36s} {sh}")
    tot = {}
    for t, k, n, sh in rows:
        a = tot.setdefault(k, [0.0, 0])
        a[0] += t
        a[1] += n
    print("--- per aten op (all shapes)")
    for k, (t, n) in sorted(tot.items(), key=lambda kv: -kv[1][0]):
        print(f"{t / 1e3:8.3f} ms {n:5d} {k}")
    ker = {}
    for e in prof.key_averages():
        t = getattr(e, "self_device_time_total", 0) or getattr(e, "self_cuda_time_total", 0)
        if t > 0 and not e.key.startswith("aten::"):
            ker[e.key] = (t, e.count)
    print("--- device kernels / non-aten (self time)")
    for k, (t, n) in sorted(ker.items(), key=lambda kv: -kv[1][0])[:60]:
        print(f"{t / 1e3:8.3f} ms {n:5d} {k[:150]}")
else:
    print(prof.key_averages().table(sort_by="self_cuda_time_total", row_limit=45, max_name_column_width=60))
