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
    ap.add_argument("--vae", action="store_true", help="the VAE encoder's conv shapes at 512² (with counts)")
    ap.add_argument("--wino", action="store_true", help="compare skp_conv3x3_wino with MIOpen (fwd, input grad)")
    args = ap.parse_args()
    if args.wino:
        return wino_vs_miopen(args)
    if args.vae:
        return vae_shapes(args)
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


def wino_vs_miopen(args):
    """(count, C, K, H) per step: VAE encoder at 512² and the UNet's 3×3 s1 layers at 64²."""
    import os, sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from stablekeypoints_amd import ops
    dev = "cuda:0"
    shapes = [(4, 128, 128, 512), (1, 128, 256, 256), (3, 256, 256, 256), (1, 256, 512, 128), (3, 512, 512, 128),
              (8, 512, 512, 64), (4, 320, 320, 64), (1, 640, 320, 64), (4, 640, 640, 32), (1, 320, 640, 32),
              (4, 1280, 1280, 16), (6, 1280, 1280, 8)]
    tm = tw = 0.0
    for (n, c, k, hw) in shapes:
        x = torch.randn(args.batch, c, hw, hw, device=dev)
        w = torch.randn(k, c, 3, 3, device=dev) / (3 * c ** 0.5)
        b = torch.randn(k, device=dev)
        fl = 2 * args.batch * hw * hw * c * k * 9
        t_m = timed(lambda: F.conv2d(x, w, b, 1, 1), iters=10)
        ok = ops.wino_eligible(args.batch, c, k, hw, hw, min_workgroups=1)
        t_w = timed(lambda: ops.Conv3x3.apply(x, w, b, None), iters=10) if ok else float("nan")
        err = float("nan")
        if ok:
            ref = F.conv2d(x.double(), w.double(), b.double(), 1, 1) if x.numel() < 2 ** 23 else None
            if ref is not None:
                err = ((ops.Conv3x3.apply(x, w, b, None).double() - ref).abs().max() / ref.abs().max()).item()
        tm += n * t_m
        tw += n * (t_w if ok else t_m)
        print(f"x{n} {c:5d}->{k:5d} {hw:4d}^2  miopen {t_m * 1e3:8.1f} us {fl / (t_m * 1e-3) / 1e12:6.1f} TF/s   "
              f"wino {t_w * 1e3:8.1f} us {fl / (t_w * 1e-3) / 1e12:6.1f} TF/s-equiv  rel.err {err:.1e}", flush=True)
        if args.bwd and ok:
            xr = x.clone().requires_grad_(True)
            out = F.conv2d(xr, w, b, 1, 1)
            g = torch.randn_like(out)
            t_mb = timed(lambda: torch.autograd.grad(out, xr, g, retain_graph=True), iters=10)
            xr2 = x.clone().requires_grad_(True)
            out2 = ops.Conv3x3.apply(xr2, w, b, None)
            t_wb = timed(lambda: torch.autograd.grad(out2, xr2, g, retain_graph=True), iters=10)
            print(f"      bwd-data miopen {t_mb * 1e3:8.1f} us   wino {t_wb * 1e3:8.1f} us", flush=True)
    print(f"total (counts applied) miopen {tm:.2f} ms  wino/miopen mix {tw:.2f} ms")


def vae_shapes(args):
    """(count, Cin, Cout, H_in, stride) of the SD VAE encoder at 512² input."""
    torch.backends.cudnn.benchmark = args.benchmark
    dev = "cuda:0"
    shapes = [(1, 3, 128, 512, 1), (4, 128, 128, 512, 1), (1, 128, 128, 512, 2), (1, 128, 256, 256, 1),
              (3, 256, 256, 256, 1), (1, 256, 256, 256, 2), (1, 256, 512, 128, 1), (3, 512, 512, 128, 1),
              (1, 512, 512, 128, 2), (8, 512, 512, 64, 1), (1, 512, 8, 64, 1)]
    total_t = total_f = 0.0
    for (n, ci, co, hw, st) in shapes:
        x = torch.randn(args.batch, ci, hw + (1 if st == 2 else 0), hw + (1 if st == 2 else 0), device=dev)
        w = torch.randn(co, ci, 3, 3, device=dev) * 0.02
        bias = torch.randn(co, device=dev)
        pad = 0 if st == 2 else 1
        if args.channels_last:
            x = x.contiguous(memory_format=torch.channels_last)
            w = w.contiguous(memory_format=torch.channels_last)
        ho = hw // st
        fl = 2 * args.batch * ho * ho * ci * co * 9
        t = timed(lambda: F.conv2d(x, w, bias, stride=st, padding=pad), iters=10)
        total_t += n * t
        total_f += n * fl
        print(f"x{n} {ci:4d}->{co:4d} {hw:4d}^2 s{st}: {t * 1e3:9.1f} us {fl / (t * 1e-3) / 1e12:6.1f} TF/s", flush=True)
    print(f"total {total_t:.2f} ms  {total_f / 1e12:.2f} TFLOP  {total_f / (total_t * 1e-3) / 1e12:.1f} TF/s")


if __name__ == "__main__":
    main()
