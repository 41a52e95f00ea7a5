"""Kernel micro-benchmark of the hot-path HIP kernels at SD-1.5 / N=500 shapes (dev tool).

Runs each kernel `--iters` times on random inputs and prints HIP-event averages; meant to be
run under `rocprofv3 --kernel-trace --stats` (or `--pmc ...`) for per-kernel breakdowns.
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from stablekeypoints_amd import ops  # noqa: E402


def timed(fn, iters):
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
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--tokens", type=int, default=500)
    ap.add_argument("--only", default="")
    args = ap.parse_args()
    dev = "cuda:0"
    N, R, H = args.tokens, 128, 8
    g = torch.Generator(device=dev).manual_seed(0)
    zs = {s: torch.randn(H, s * s, N, device=dev, generator=g) * 2 for s in (16, 32)}
    attn = {s: ops.capture_attn(zs[s], s, R) for s in (16, 32)}
    # four DISTINCT layers (repeating one tensor would let the 256 MB L3 serve re-reads)
    layers = [ops.capture_attn(zs[16] * (1 + 0.1 * i), 16, R) for i in range(3)] + [attn[32]]
    dmap = torch.randn(N, R * R, device=dev, generator=g)
    gb = dmap.t().unsqueeze(0).expand(H, R * R, N)
    # the bench's backward: 2 images x H heads, per-image token-major map gradient (CaptureMaps)
    zb2 = {s: torch.randn(2 * H, s * s, N, device=dev, generator=g) * 2 for s in (16, 32)}
    gmap = torch.randn(2, N, R, R, device=dev, generator=g)
    bstr = (N * R * R, 1, R * R)
    res = {}
    todo = args.only.split(",") if args.only else ["fwd16", "fwd32", "agg", "bwd16", "bwd32", "bwd16b2", "bwd32b2", "bwd16_dense"]
    for name in todo:
        if name == "fwd16":
            res[name] = timed(lambda: ops.capture_attn(zs[16], 16, R), args.iters)
        elif name == "fwd32":
            res[name] = timed(lambda: ops.capture_attn(zs[32], 32, R), args.iters)
        elif name == "agg":
            res[name] = timed(lambda: ops.aggregate(layers), args.iters)
        elif name == "bwd16":
            res[name] = timed(lambda: ops.capture_bwd(zs[16], 16, R, gb), args.iters)
        elif name == "bwd32":
            res[name] = timed(lambda: ops.capture_bwd(zs[32], 32, R, gb), args.iters)
        elif name in ("bwd16b2", "bwd32b2", "bwd16b2s", "bwd32b2s"):
            sz = 16 if name.startswith("bwd16") else 32
            st = None
            if name.endswith("s"):   # with the forward's per-pixel softmax stats (the bench's path)
                from stablekeypoints_amd._lib import call, ptr, stream
                st = torch.empty(2 * H, R * R, 2, device=dev)
                scratch = torch.empty(2 * H, R * R, N, device=dev)
                call("skp_capture_fwd", ptr(zb2[sz]), 2 * H, sz, N, R, ptr(scratch), ptr(st), stream(dev))
                del scratch
            res[name] = timed(lambda: ops.capture_bwd(zb2[sz], sz, R, gmap, 0.03125, H, bstr, stats=st), args.iters)
        elif name in ("maps8", "maps8_old", "maps8_s16", "maps8_s32"):   # fused capture + per-image aggregate, bench shape
            # (_s16 / _s32: only the bench's s = 16 layers / its s = 32 layer, for per-layer PMC passes)
            sizes = {"maps8_s16": (16, 16, 16), "maps8_s32": (32,)}.get(name, (16, 16, 16, 32))
            z8 = [torch.randn(8 * H, s * s, N, device=dev, generator=g) * 2 for s in sizes]
            ops.FUSED_MAPS = name != "maps8_old"
            with torch.no_grad():
                res[name] = timed(lambda: ops.capture_maps(z8, sizes, 8, R), args.iters)
            ops.FUSED_MAPS = True
            del z8
        elif name in ("mapsbwd8", "mapsbwd8_old"):   # fused backward vs per-layer capture_bwd, bench shape
            sizes = (16, 16, 16, 32)
            z8 = [(torch.randn(8 * H, s * s, N, device=dev, generator=g) * 2).requires_grad_(True) for s in sizes]
            ops.FUSED_MAPS = True
            maps = ops.capture_maps(z8, sizes, 8, R)
            gm = torch.randn_like(maps)
            ops.FUSED_MAPS = name == "mapsbwd8"
            res[name] = timed(lambda: torch.autograd.grad(maps, z8, gm, retain_graph=True), args.iters)
            ops.FUSED_MAPS = True
            del z8, maps, gm
        elif name in ("mapssel8", "mapssel8_dense", "mapssel8_s16", "mapssel8_s32"):
            # sparse backward of 10 selected rows per image, bench shape (_s16 / _s32: one layer class)
            sizes = {"mapssel8_s16": (16, 16, 16), "mapssel8_s32": (32,)}.get(name, (16, 16, 16, 32))
            z8 = [(torch.randn(8 * H, s * s, N, device=dev, generator=g) * 2).requires_grad_(True) for s in sizes]
            ops.SEL_BWD = name != "mapssel8_dense"
            cm = ops.CapturedMaps(z8, sizes, 8, R)
            rows = [torch.randperm(N, device=dev, generator=g)[:10] for _ in range(8)]
            out = cm.select(rows)
            gsel = torch.randn_like(out)
            res[name] = timed(lambda: torch.autograd.grad(out, z8, gsel, retain_graph=True), args.iters)
            ops.SEL_BWD = True
            del z8, cm, out, gsel
        elif name == "sum1g":   # read-bandwidth reference: torch reduction over a fresh 1 GiB tensor
            big = torch.empty(256 * 1024 * 1024, device=dev).normal_()
            res[name] = timed(lambda: big.sum(), args.iters)
            res[name + "_GBs"] = big.numel() * 4 / (res[name] * 1e-3) / 1e9 / 1e3
        elif name == "copy1g":
            big = torch.empty(256 * 1024 * 1024, device=dev).normal_()
            dst = torch.empty_like(big)
            res[name] = timed(lambda: dst.copy_(big), args.iters)
            res[name + "_GBs"] = 2 * big.numel() * 4 / (res[name] * 1e-3) / 1e9 / 1e3
        elif name.startswith("gemm"):   # capture logits q kᵀ and its two gradients at s=16/32, bench batch 8
            sz = 16 if name.endswith("16") else 32
            d = 160 if sz == 16 else 80
            q = torch.randn(8 * H, sz * sz, d, device=dev, generator=g)
            k = torch.randn(8 * H, N, d, device=dev, generator=g)
            dz = torch.randn(8 * H, sz * sz, N, device=dev, generator=g)
            t_f = timed(lambda: ops.bgemm(q, k.transpose(1, 2), 0.1), args.iters)
            t_q = timed(lambda: ops.bgemm(dz, k, 0.1), args.iters)
            t_k = timed(lambda: ops.bgemm(dz.transpose(1, 2), q, 0.1), args.iters)
            t_ref = timed(lambda: torch.bmm(q, k.transpose(1, 2)), args.iters)
            fl = 2 * 8 * H * sz * sz * N * d
            for nm, t in (("fwd", t_f), ("dq", t_q), ("dk", t_k), ("torch_fwd", t_ref)):
                res[f"{name}_{nm}"] = t
                res[f"{name}_{nm}_TFs"] = fl / (t * 1e-3) / 1e12 / 1e3
        elif name in ("kl", "argmax", "fps", "sharp", "equiv", "entropy"):
            maps = torch.rand(N, R, R, device=dev, generator=g) ** 8   # peaked, attention-map-like
            A10 = maps[:10].contiguous()
            At10 = maps[10:20].contiguous()
            th = torch.tensor([[0.9, -0.1, 0.05], [0.1, 0.9, -0.02]], device=dev)
            cand = torch.arange(25, device=dev)
            fn = {"kl": lambda: ops.find_top_k_gaussian(maps, 25, sigma=2.0),
                  "entropy": lambda: ops.entropy_sort(maps, 25),
                  "argmax": lambda: ops.find_max_pixel(maps),
                  "fps": lambda: ops.furthest_point_sampling(maps, 10, cand),
                  "sharp": lambda: ops.sharpening_loss(A10, 2.0),
                  "equiv": lambda: ops.equivariance_loss_single(A10, At10, th)}[name]
            res[name] = timed(fn, args.iters)
        elif name in ("kl4", "kl4_s2", "kl8_256"):   # the A8 KL ranking of a pass's images, one launch
            nb, rr = (8, 256) if name == "kl8_256" else (4, R)
            m4 = torch.rand(nb, N, rr, rr, device=dev, generator=g) ** 8
            ns = 2 if name == "kl4_s2" else 1
            res[name] = timed(lambda: ops.find_top_k_gaussian_batch(m4, 25, sigma=2.0, num_subjects=ns), args.iters)
            res[name + "_GBs"] = m4.numel() * 4 / (res[name] * 1e-3) / 1e9 / 1e3
            del m4
        elif name in ("sel4", "sel4_r05"):   # a pass's selection chain: 4 images' KL keys, 25 candidates, FPS 10
            m4 = torch.rand(4, N, R, R, device=dev, generator=g) ** 8
            mt4 = torch.rand(4, N, R, R, device=dev, generator=g) ** 8
            if name == "sel4":   # r06: KL → rank + argmax → FPS
                fn = lambda: ops.gaussian_fps_batch(m4, mt4, 25, 10, sigma=2.0)
            else:                # r05: KL → rank → argmax → FPS
                fn = lambda: ops.furthest_point_sampling_batch(mt4, 10, ops.find_top_k_gaussian_batch(m4, 25, sigma=2.0))
            res[name] = timed(fn, args.iters)
            del m4, mt4
        elif name == "bwd16_dense":
            res[name] = timed(lambda: ops.capture_bwd(zs[16], 16, R, attn[16]), args.iters)
    agg_bytes = (4 * H * R * R * N + N * R * R) * 4
    for k, v in res.items():
        extra = f"  {agg_bytes / (v * 1e-3) / 1e9:.0f} GB/s" if k == "agg" else ""
        print(f"{k:12s} {v * 1e3:9.1f} us{extra}", flush=True)


if __name__ == "__main__":
    main()
