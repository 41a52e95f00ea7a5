"""Host enqueue time vs GPU time of the bench's optimiser step (dev tool): if the host needs about as
long to issue a step's kernels as the GPU needs to run them, the GPU waits on the host.

    python tools/host_time.py [--steps 6]
"""
import argparse
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from stablekeypoints_amd.datasets import SyntheticDataset  # noqa: E402
from stablekeypoints_amd.optimize import TokenOptimizer  # noqa: E402
from stablekeypoints_amd.optimize_token import load_ldm  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--steps", type=int, default=6)
ap.add_argument("--prefetch", type=int, default=2)
args = ap.parse_args()
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
c = [0]


def batch(k):
    return [imgs[(k + i) % 16] for i in range(4)]


ORDER = os.environ.get("HOST_ORDER", "mid")


def step():
    t = [time.perf_counter()]
    opt.prefetch(batch(c[0]))
    if ORDER == "before":
        for d in range(1, args.prefetch + 1):
            opt.prefetch(batch(c[0] + 4 * d))
    t.append(time.perf_counter())
    opt.micro_steps(batch(c[0]), prefetch=[batch(c[0] + 4 * d) for d in range(1, args.prefetch + 1)]
                    if ORDER == "mid" else ())
    t.append(time.perf_counter())
    if ORDER == "after":
        for d in range(1, args.prefetch + 1):
            opt.prefetch(batch(c[0] + 4 * d))
    opt.optimizer_step()
    t.append(time.perf_counter())
    c[0] += 4
    return t


for _ in range(2):
    step()
torch.cuda.synchronize()
ev = [torch.cuda.Event(enable_timing=True) for _ in range(args.steps + 1)]
ev[0].record()
t0 = time.perf_counter()
host = []
for i in range(args.steps):
    t = step()
    host.append((t[1] - t[0], t[2] - t[1], t[3] - t[2]))
    ev[i + 1].record()
t_host = time.perf_counter() - t0
torch.cuda.synchronize()
t_all = time.perf_counter() - t0
for i, (a, b, cc) in enumerate(host):
    print(f"step {i}: host prefetch-before {a * 1e3:6.1f} ms, micro_steps {b * 1e3:6.1f} ms, "
          f"prefetch-after + adam {cc * 1e3:5.1f} ms; "
          f"GPU (main-stream events) {ev[i].elapsed_time(ev[i + 1]):6.1f} ms", flush=True)
print(f"host issued {args.steps} steps in {t_host * 1e3:.1f} ms; all done after {t_all * 1e3:.1f} ms", flush=True)
