"""Where do the step's strided copies / adds / fills come from?  Runs one token-opt pass (4 images +
warps, batch-8 forward + backward) under a TorchDispatchMode that records every copy-like aten call
with its output size, the input strides and its call site: the nearest repo frame of the Python
stack (forward, custom-Function backward) or the autograd node running it (built-in backward).
Prints the sites by bytes moved (dev tool).

    python tools/copy_sites.py [--rows 60] [--min-mb 1]
"""
import argparse
import collections
import os
import sys
import traceback

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from torch.utils._python_dispatch import TorchDispatchMode

from stablekeypoints_amd.datasets import SyntheticDataset
from stablekeypoints_amd.optimize import TokenOptimizer
from stablekeypoints_amd.optimize_token import load_ldm

ap = argparse.ArgumentParser()
ap.add_argument("--rows", type=int, default=60)
ap.add_argument("--min-mb", type=float, default=1.0)
OPT = ap.parse_args()

WATCH = ("copy_", "clone", "_to_copy", "cat", "add", "mul", "fill_", "zero_", "sub", "div", "sum", "where",
         "index", "scatter", "new_zeros", "zeros")
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def site():
    fr = [f for f in traceback.extract_stack()[:-3] if f.filename.startswith(REPO) and "tools/" not in f.filename]
    node = torch._C._current_autograd_node()
    where = " <- ".join(f"{os.path.relpath(f.filename, REPO)}:{f.lineno}" for f in fr[-3:][::-1])
    if node is not None:
        where = f"bwd[{node.name()}] " + where
    return where


class Rec(TorchDispatchMode):
    def __init__(self):
        super().__init__()
        self.rows = collections.defaultdict(lambda: [0, 0.0])

    def __torch_dispatch__(self, func, types, args=(), kwargs=None):
        out = func(*args, **(kwargs or {}))
        name = func.__name__
        if any(w in name for w in WATCH):
            t = out[0] if isinstance(out, (tuple, list)) and out and torch.is_tensor(out[0]) else out
            if torch.is_tensor(t) and t.is_cuda:
                mb = t.numel() * t.element_size() / 2 ** 20
                if mb >= OPT.min_mb:
                    ins = [a for a in args if torch.is_tensor(a)]
                    sh = tuple(t.shape)
                    st = tuple(tuple(a.stride()) for a in ins[:2])
                    key = (name, sh, st, site())
                    r = self.rows[key]
                    r[0] += 1
                    r[1] += mb
        return out


dev = torch.device("cuda:0")
ldm, ctls, _ = load_ldm(dev, "random", feature_upsample_res=128)
torch.manual_seed(0)
ctx = torch.randn(1, 500, 768).to(dev)
opt = TokenOptimizer(ldm, ctls, ctx, accum=4, device=dev)
data = SyntheticDataset(n=8, size=512)
imgs = [data[i]["img"][None].to(dev) for i in range(8)]
opt.micro_steps(imgs[:4])
opt.optimizer_step()
torch.cuda.synchronize()
opt.prefetch(imgs[4:])
rec = Rec()
with rec:
    opt.micro_steps(imgs[4:], prefetch=[imgs[:4]])
torch.cuda.synchronize()
tot = sum(r[1] for r in rec.rows.values())
print(f"copy-like aten outputs >= {OPT.min_mb} MB in one pass (+ the next pass's VAE prefetch): {tot:.0f} MB")
for (name, sh, st, where), (n, mb) in sorted(rec.rows.items(), key=lambda kv: -kv[1][1])[:OPT.rows]:
    print(f"{mb:9.1f} MB {n:4d} {name:22s} {str(sh):26s} {str(st)[:60]:60s} {where}")
