"""cProfile of the host side of one bench optimiser step after warm-up (dev tool): where the Python
time goes between kernel launches.

    python tools/host_profile.py [--sort tottime] [--rows 40]
"""
import argparse
import cProfile
import os
import pstats
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from stablekeypoints_amd.datasets import SyntheticDataset  # noqa: E402
from stablekeypoints_amd.optimize import TokenOptimizer  # noqa: E402
from stablekeypoints_amd.optimize_token import load_ldm  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--sort", default="tottime")
ap.add_argument("--rows", type=int, default=40)
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


def step():
    opt.prefetch(batch(c[0]))
    opt.micro_steps(batch(c[0]))
    for d in (1, 2):
        opt.prefetch(batch(c[0] + 4 * d))
    opt.optimizer_step()
    c[0] += 4


for _ in range(3):
    step()
torch.cuda.synchronize()
t0 = time.perf_counter()
pr = cProfile.Profile()
pr.enable()
step()
pr.disable()
t1 = time.perf_counter()
torch.cuda.synchronize()
t2 = time.perf_counter()
print(f"host {1e3 * (t1 - t0):.1f} ms (profiled), GPU done after {1e3 * (t2 - t0):.1f} ms", flush=True)
pstats.Stats(pr).sort_stats(args.sort).print_stats(args.rows)
