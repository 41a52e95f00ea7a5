"""Dev tool: time the SD-1.5 UNet/VAE 3x3 convolutions (--batch, default 2) under MIOpen settings.

usage: python tools/conv_probe.py [--benchmark] [--channels-last]
(set MIOPEN_FIND_MODE etc. in the environment to compare find modes)
"""
import argparse
import torch
import torch.nn.functional as F


def timed(fn, iters=20):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--benchmark", action="store_true")
    ap.add_argument("--channels-last", action="store_true")
    ap.add_argument("--bwd", action="store_true")
    ap.add_argument("--batch", type=int, default=2)
    args = ap.parse_args()
    torch.backends.cudnn.benchmark = args.benchmark
    dev = "cuda:0"
    for (hw, c) in [(64, 320), (32, 640), (16, 1280), (64, 640), (128, 512), (256, 256)]:
        x = torch.randn(args.batch, c, hw, hw, device=dev)
        w = torch.randn(c, c, 3, 3, device=dev) * 0.02
        bias = torch.randn(c, device=dev)
        if args.channels_last:
            x = x.contiguous(memory_format=torch.channels_last)
            w = w.contiguous(memory_format=torch.channels_last)
        fl = 2 * args.batch * hw * hw * c * c * 9
        t = timed(lambda: F.conv2d(x, w, bias, padding=1))
        line = f"fwd {hw:4d}^2 c={c:5d}: {t * 1e3:8.1f} us  {fl / (t * 1e-3) / 1e12:6.1f} TF/s"
        if args.bwd:
            xr = x.clone().requires_grad_(True)
            out = F.conv2d(xr, w, bias, padding=1)
            g = torch.randn_like(out)
            tb = timed(lambda: torch.autograd.grad(out, xr, g, retain_graph=True))
            line += f"   bwd-data {tb * 1e3:8.1f} us {fl / (tb * 1e-3) / 1e12:6.1f} TF/s"
        print(line, flush=True)


if __name__ == "__main__":
    main()
