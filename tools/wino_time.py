"""Dev tool: time skp_conv3x3_wino forward on a few shapes (TF/s-equivalent of the direct conv).

usage: python tools/wino_time.py [--shapes B,C,K,HW;...]  (timing-probe builds: tools/build_variant.sh with -DSKP_WINO_DEBUG=… / -DSKP_WINO2_DEBUG=…)
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from stablekeypoints_amd import ops

ap = argparse.ArgumentParser()
ap.add_argument("--shapes", default="8,128,128,512;8,512,512,128;8,512,512,64;8,320,320,64;8,640,640,32;8,1280,1280,16")
ap.add_argument("--iters", type=int, default=10)
ap.add_argument("--residual", action="store_true", help="bias + residual epilogue (the resnet conv2 form)")
a = ap.parse_args()
for s in a.shapes.split(";"):
    B, C, K, HW = map(int, s.split(","))
    x = torch.randn(B, C, HW, HW, device="cuda:0")
    w = torch.randn(K, C, 3, 3, device="cuda:0") / (3 * C ** 0.5)
    b = torch.randn(K, device="cuda:0") if a.residual else None
    r = torch.randn(B, K, HW, HW, device="cuda:0") if a.residual else None
    f = lambda: ops._wino_conv(x, w, False, b, r, K)
    f()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(a.iters):
        f()
    e1.record()
    torch.cuda.synchronize()
    t = e0.elapsed_time(e1) / a.iters
    fl = 2 * B * HW * HW * C * K * 9
    print(f"{B}x{C}->{K} {HW}^2: {t * 1e3:8.1f} us  {fl / (t * 1e-3) / 1e12:6.1f} TF/s-equiv  "
          f"({fl / 4 / (t * 1e-3) / 1e12:5.1f} TF/s MFMA)", flush=True)
