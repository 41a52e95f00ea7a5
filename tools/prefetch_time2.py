"""Host time of TokenOptimizer.prefetch's pieces inside the real step (mid-pass prefetch, steady state;
dev tool)."""
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
import gc
gc.collect()
gc.freeze()
torch.manual_seed(0)
ctx = torch.randn(1, 500, 768).to(dev)
opt = TokenOptimizer(ldm, ctls, ctx, accum=4, device=dev)
data = SyntheticDataset(n=16, size=512)
imgs = [data[i]["img"][None].to(dev) for i in range(16)]
log = []


def prefetch(self, images):
    key = tuple(id(t) for t in images)
    if any(r[0] == key for r in self._prefetched):
        return
    if self._side is None:
        self._side = torch.cuda.Stream(device=self.device)
    t = [time.perf_counter()]
    batch = torch.cat(list(images))
    thetas = self.draw_thetas(len(images))
    main = torch.cuda.current_stream(self.device)
    self._side.wait_stream(main)
    t.append(time.perf_counter())
    with torch.cuda.stream(self._side), torch.no_grad():
        batch.record_stream(self._side)
        thd = _upload(thetas.float(), self.device)
        t.append(time.perf_counter())
        transformed = ops.affine_warp(batch, thd)
        t.append(time.perf_counter())
        both = torch.cat([batch, transformed])
        t.append(time.perf_counter())
        lat = ptp_utils.image2latent(self.ldm, both, self.device)
        t.append(time.perf_counter())
        ev = torch.cuda.Event()
        ev.record(self._side)
    self._prefetched.append((key, thetas, lat, ev))
    t.append(time.perf_counter())
    log.append([1e3 * (b - a) for a, b in zip(t, t[1:])])


TokenOptimizer.prefetch = prefetch
c = [0]


def batch(k):
    return [imgs[(k + i) % 16] for i in range(4)]


for i in range(7):
    opt.prefetch(batch(c[0]))
    opt.micro_steps(batch(c[0]), prefetch=[batch(c[0] + 4)])
    opt.optimizer_step()
    c[0] += 4
torch.cuda.synchronize()
for i, l in enumerate(log):
    print(f"prefetch {i}: " + ", ".join(f"{n} {v:6.2f}" for n, v in zip(["cat+thetas", "upload", "warp", "cat2", "vae", "event"], l)) + " ms", flush=True)
