"""Dev tool: run one skp_conv3x3_wino shape a few times (for rocprofv3 PMC passes)."""
import os, sys, argparse
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from stablekeypoints_amd import ops

ap = argparse.ArgumentParser()
ap.add_argument("--shape", default="8,128,128,512")
ap.add_argument("--iters", type=int, default=5)
a = ap.parse_args()
B, C, K, HW = map(int, a.shape.split(","))
x = torch.randn(B, C, HW, HW, device="cuda:0")
w = torch.randn(K, C, 3, 3, device="cuda:0") / (3 * C ** 0.5)
for _ in range(a.iters):
    y = ops.Conv3x3.apply(x, w, None, None)
torch.cuda.synchronize()
print("ok", y.shape)
