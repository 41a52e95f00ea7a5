"""Dev probe: the UNet's 8² × 1280 3×3 convolutions — Winograd v1 (split-K) vs im2col + one
hipBLASLt GEMM vs MIOpen, forward shapes C = 1280 / 2560 → K = 1280, batch 8."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import torch.nn.functional as F
from stablekeypoints_amd import ops

dev = "cuda:0"
if os.environ.get("TUNE") == "1":
    t = torch.cuda.tunable
    t.enable(True); t.tuning_enable(True); t.set_max_tuning_duration(30)
    t.set_filename(os.path.join(os.environ.get("GRAFT_REPO_ROOT", "."), "gpurun_out", "conv8_tune%d.csv"))


def timed(fn, iters=50):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters):
        fn()
    b.record(); torch.cuda.synchronize()
    return a.elapsed_time(b) / iters * 1e3


def im2col_bmm(x, wm, bias):
    cols = F.unfold(x, 3, padding=1)                      # (B, C·9, HW)
    return torch.baddbmm(bias.view(1, -1, 1), wm.expand(x.shape[0], *wm.shape), cols)


def im2col_mm(x, wm, bias):
    B, C, H, W = x.shape
    cols = F.unfold(x, 3, padding=1).permute(1, 0, 2).reshape(C * 9, B * H * W)
    y = torch.addmm(bias.view(-1, 1), wm, cols)            # (K, B·HW)
    return y.view(-1, B, H * W).permute(1, 0, 2)


def im2col_mm_t(x, wm, bias):
    # rows = pixels: (B·HW, C·9) @ (C·9, K) -> (B·HW, K), then to NCHW
    B, C, H, W = x.shape
    cols = F.unfold(x, 3, padding=1).transpose(1, 2).reshape(B * H * W, C * 9)
    y = torch.addmm(bias, cols, wm.t())
    return y.view(B, H * W, -1).transpose(1, 2)


for C in (1280, 2560):
    K, B, H = 1280, 8, 8
    g = torch.Generator(device=dev).manual_seed(C)
    x = torch.randn(B, C, H, H, device=dev, generator=g)
    w = torch.randn(K, C, 3, 3, device=dev, generator=g) * (C * 9) ** -0.5
    bias = torch.randn(K, device=dev, generator=g)
    wm = w.reshape(K, C * 9).contiguous()
    ref = F.conv2d(x.double(), w.double(), bias.double(), 1, 1)
    res = {}
    for name, fn in (("wino_v1", lambda: ops.conv3x3(x, w, bias)), ("miopen", lambda: F.conv2d(x, w, bias, 1, 1)),
                     ("im2col_bmm", lambda: im2col_bmm(x, wm, bias)), ("im2col_mm", lambda: im2col_mm(x, wm, bias)),
                     ("im2col_mm_t", lambda: im2col_mm_t(x, wm, bias))):
        out = fn().reshape(B, K, H, H)
        err = ((out.double() - ref).abs().max() / ref.abs().max()).item()
        res[name] = (timed(fn), err)
    fl = 2 * B * H * H * C * K * 9
    print(f"C={C}: " + "  ".join(f"{k} {t:.1f} us ({fl / t / 1e6:.0f} TF/s, rel err {e:.1e})" for k, (t, e) in res.items()), flush=True)
