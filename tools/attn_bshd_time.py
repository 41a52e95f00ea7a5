"""A/B timing of one UNet attention call on the (B, S, H·d) projections (ops.attention_heads) vs the
head-permuting path (reshape_heads_to_batch_dim → ops.math_attention → reshape_batch_dim_to_heads),
forward + backward, at the SD-1.5 bench shapes (dev tool).

    python tools/attn_bshd_time.py [--iters 20]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from stablekeypoints_amd import ops  # noqa: E402


def heads(t, H):
    b, s, c = t.shape
    return t.reshape(b, s, H, c // H).permute(0, 2, 1, 3).reshape(b * H, s, c // H)


def merge(t, H):
    bh, s, d = t.shape
    return t.reshape(bh // H, H, s, d).permute(0, 2, 1, 3).reshape(bh // H, s, d * H)


def timed(fn, iters):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / iters * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=20)
    args = ap.parse_args()
    dev = "cuda:0"
    g = torch.Generator(device=dev).manual_seed(0)
    B, H = 8, 8
    ap_only = os.environ.get("ATTN_ONLY", "")
    for name, S, L, C, shared in (("64x64 self", 4096, 4096, 320, False), ("64x64 cross", 4096, 500, 320, True),
                                  ("32x32 self", 1024, 1024, 640, False)):
        if ap_only and ap_only not in name:
            continue
        d = C // H
        q = torch.randn(B, S, C, device=dev, generator=g).requires_grad_(True)
        k1 = torch.randn(1 if shared else B, L, C, device=dev, generator=g).requires_grad_(True)
        v1 = torch.randn(1 if shared else B, L, C, device=dev, generator=g).requires_grad_(True)
        go = torch.randn(B, S, C, device=dev, generator=g)
        scale = d ** -0.5

        def kv():
            return (k1.expand(B, L, C), v1.expand(B, L, C)) if shared else (k1, v1)

        def bshd():
            k, v = kv()
            out = ops.attention_heads(q, k, v, H, scale)
            torch.autograd.backward(out, go)

        def perm():
            k, v = kv()
            out = merge(ops.math_attention(heads(q, H), heads(k, H), heads(v, H), scale), H)
            torch.autograd.backward(out, go)

        with torch.no_grad():
            def bshd_ng():
                k, v = kv()
                ops.attention_heads(q, k, v, H, scale)

            def perm_ng():
                k, v = kv()
                merge(ops.attention_nograd(heads(q, H), heads(k, H), heads(v, H), scale), H)
            t_ng = (timed(bshd_ng, args.iters), timed(perm_ng, args.iters))
        k, v = kv()
        res = [timed(bshd, args.iters) if ops.attention_heads(q, k, v, H, scale) is not None else float("nan"),
               timed(perm, args.iters)]
        print(f"{name:12s} d={d:3d}  fwd+bwd: bshd {res[0]:8.1f} us  permute {res[1]:8.1f} us   "
              f"no-grad fwd: bshd {t_ng[0]:8.1f} us  permute {t_ng[1]:8.1f} us", flush=True)


if __name__ == "__main__":
    main()
