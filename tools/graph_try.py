"""Feasibility / speed probe: the token-opt pass (capture forward, selection, losses, backward into
the embedding) captured as ONE HIP graph and replayed, vs eager (dev tool)."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from stablekeypoints_amd import ops, ptp_utils  # noqa: E402
from stablekeypoints_amd.datasets import SyntheticDataset  # noqa: E402
from stablekeypoints_amd.optimize import TokenOptimizer  # noqa: E402
from stablekeypoints_amd.optimize_token import load_ldm  # noqa: E402

dev = torch.device("cuda:0")
TINY = "--tiny" in sys.argv
torch.manual_seed(0)
if TINY:       # the GPU tests' toy SD (tests/test_gpu_graph.py)
    from stablekeypoints_amd.sd import TINY_CONFIG, TINY_IMAGE
    ldm, ctls, _ = load_ldm(dev, "tiny", feature_upsample_res=32, config=TINY_CONFIG)
    ctx = torch.randn(1, 16, 32).to(dev)
    opt = TokenOptimizer(ldm, ctls, ctx, top_k=4, furthest_point_num_samples=8, accum=4, device=dev)
else:
    ldm, ctls, _ = load_ldm(dev, "random", feature_upsample_res=128)
    ctx = torch.randn(1, 500, 768).to(dev)
    opt = TokenOptimizer(ldm, ctls, ctx, accum=4, device=dev)
data = SyntheticDataset(n=16, size=TINY_IMAGE if TINY else 512)
imgs = [data[i]["img"][None].to(dev) for i in range(16)]
k = 4
with torch.no_grad():
    batch = torch.cat(imgs[:4])
    th = opt.draw_thetas(4)
    tr = ops.affine_warp(batch, th.to(dev))
    lat = ptp_utils.image2latent(ldm, torch.cat([batch, tr]), dev)
static_in = lat.clone()
opt.transform.last_params = {"theta": th.float()}
static_thinv = opt.transform.theta_inverse().to(dev)


def body():
    got = ptp_utils.run_and_find_attn_per_image(ldm, static_in, opt.context, noise_level=-1, device=dev,
                                                layers=(0, 1, 2, 3), controllers=opt.controllers, stacked=True,
                                                captured=True)[0]
    maps = got.maps
    sel = [opt._select(maps[i], maps[k + i]) for i in range(k)]
    rows = got.select(sel + sel)
    n = rows.shape[0] // 2
    A, At = rows[:n], rows[n:]
    total, off = 0.0, 0
    for i, idx in enumerate(sel):
        m = idx.numel()
        loss, eq, sh = opt._losses(A[off:off + m], At[off:off + m], i, static_thinv[i])
        off += m
        total = total + loss
    (total / 4).backward()
    return sel, total


s = torch.cuda.Stream()
s.wait_stream(torch.cuda.current_stream())
with torch.cuda.stream(s):
    for _ in range(3):
        opt.optimizer.zero_grad(set_to_none=True)
        body()
torch.cuda.current_stream().wait_stream(s)
torch.cuda.synchronize()


def timed(fn, n=5):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / n * 1e3


def eager():
    opt.optimizer.zero_grad(set_to_none=True)
    body()


print(f"eager pass: {timed(eager):.1f} ms", flush=True)
g = torch.cuda.CUDAGraph()
opt.optimizer.zero_grad(set_to_none=True)
try:
    with torch.cuda.graph(g):
        sel_s, total_s = body()
except Exception as e:  # report what breaks capture
    print("CAPTURE FAILED:", type(e).__name__, str(e)[:2000], flush=True)
    raise
torch.cuda.synchronize()
print("captured; grad", opt.context.grad is not None, flush=True)
print(f"graph replay: {timed(g.replay):.1f} ms", flush=True)
g.replay()
torch.cuda.synchronize()
gg = opt.context.grad.clone()
sg = [x.clone() for x in sel_s]
eager()
torch.cuda.synchronize()
print("sel equal:", all(torch.equal(a, b) for a, b in zip(sg, [x for x in sel_s])), flush=True)
