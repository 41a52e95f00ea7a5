"""Host time of the pieces of TokenOptimizer.prefetch while the GPU is busy with a UNet pass
(dev tool): which host call blocks."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from stablekeypoints_amd import ops, ptp_utils  # noqa: E402
from stablekeypoints_amd.datasets import SyntheticDataset  # noqa: E402
from stablekeypoints_amd.optimize import TokenOptimizer, _upload  # noqa: E402
from stablekeypoints_amd.optimize_token import load_ldm  # noqa: E402

dev = torch.device("cuda:0")
ldm, ctls, _ = load_ldm(dev, "random", feature_upsample_res=128)
torch.manual_seed(0)
ctx = torch.randn(1, 500, 768).to(dev)
opt = TokenOptimizer(ldm, ctls, ctx, accum=4, device=dev)
data = SyntheticDataset(n=16, size=512)
imgs = [data[i]["img"][None].to(dev) for i in range(16)]
side = torch.cuda.Stream(device=dev)
for it in range(6):
    busy = torch.randn(8192, 8192, device=dev)
    for _ in range(20):   # ~tens of ms of queued main-stream work
        busy = busy @ busy * 1e-4
    t = [time.perf_counter()]
    batch = torch.cat(imgs[:4])
    t.append(time.perf_counter())
    th = opt.draw_thetas(4)
    t.append(time.perf_counter())
    side.wait_stream(torch.cuda.current_stream(dev))
    with torch.cuda.stream(side), torch.no_grad():
        batch.record_stream(side)
        thd = _upload(th.float(), dev)
        t.append(time.perf_counter())
        tr = ops.affine_warp(batch, thd)
        t.append(time.perf_counter())
        lat = ptp_utils.image2latent(ldm, torch.cat([batch, tr]), dev)
        t.append(time.perf_counter())
    names = ["cat", "thetas", "upload", "warp", "vae"]
    print(f"iter {it}: " + ", ".join(f"{n} {1e3 * (b - a):6.2f} ms" for n, a, b in zip(names, t, t[1:])), flush=True)
    torch.cuda.synchronize()
