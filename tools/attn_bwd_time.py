"""Dev tool: time the math-attention backward's score-gradient paths at the 64²-token shape."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from stablekeypoints_amd import ops
from stablekeypoints_amd._lib import call, ptr, stream

dev = "cuda:0"
BH, S, L, d = 64, 4096, 4096, 40
g = torch.Generator(device=dev).manual_seed(0)
q = torch.randn(BH, S, d, device=dev, generator=g)
k = torch.randn(BH, L, d, device=dev, generator=g)
v = torch.randn(BH, L, d, device=dev, generator=g)
p = ops.attention_probs(q, k, d ** -0.5)
out = torch.bmm(p, v)
dout = torch.randn_like(out)


def timed(fn, iters=5):
    fn(); torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters):
        fn()
    b.record(); torch.cuda.synchronize()
    return a.elapsed_time(b) / iters


def old():
    ds = torch.bmm(dout, v.transpose(1, 2))
    call("skp_softmax_bwd", ptr(p), ptr(ds), BH * S, L, 0.158, stream(dev))
    return ds


ds_new = torch.empty_like(p)


def new():
    D = (dout * out).sum(-1)
    call("skp_attn_dscore", ptr(p), ptr(dout), ptr(v), ptr(D), ptr(ds_new), BH, S, L, d, 0.158, stream(dev))
    return ds_new


print(f"old (dP GEMM + softmax_bwd): {timed(old):.3f} ms   fused dscore: {timed(new):.3f} ms")
f_old = lambda: torch.bmm(ops.attention_probs(q, k, d ** -0.5), v)
f_new = lambda: ops.attention_nograd(q, k, v, d ** -0.5)
print(f"forward: scores+softmax+PV {timed(f_old):.3f} ms   fused online-softmax {timed(f_new):.3f} ms   "
      f"max diff {(f_old() - f_new()).abs().max().item():.2e}")
a, b = old(), new()
print("max rel diff", ((a - b).abs().max() / a.abs().max()).item())

dv_, dk_ = torch.empty_like(v), torch.empty_like(k)


def full_unfused():
    dv = torch.bmm(p.transpose(1, 2), dout)
    ds = new()
    return torch.bmm(ds, k), torch.bmm(ds.transpose(1, 2), q), dv


def full_fused():
    D = (dout * out).sum(-1)
    call("skp_attn_bwd_kv", ptr(p), ptr(dout), ptr(q), ptr(v), ptr(D), ptr(ds_new), ptr(dv_), ptr(dk_),
         BH, S, L, d, 0.158, stream(dev))
    return torch.bmm(ds_new, k), dk_, dv_


print(f"full backward: unfused {timed(full_unfused):.3f} ms   fused dS/dV/dK {timed(full_fused):.3f} ms")
a, b = full_unfused(), full_fused()
print("max rel diff dq/dk/dv", [((x - y).abs().max() / x.abs().max()).item() for x, y in zip(a, b)])

stats = torch.empty(BH, S, 2, device=dev)
o_fl = torch.empty_like(q)
ds_fl, dv_fl, dk_fl = torch.empty_like(p), torch.empty_like(v), torch.empty_like(k)


def flash_fwd():
    call("skp_attn_fwd", ptr(q), ptr(k), ptr(v), ptr(o_fl), ptr(stats), BH, S, L, d, d ** -0.5, stream(dev))


def flash_bwd():
    D = (dout * o_fl).sum(-1)
    call("skp_attn_bwd_flash", ptr(q), ptr(k), ptr(v), ptr(dout), ptr(stats), ptr(D), ptr(ds_fl), ptr(dv_fl),
         ptr(dk_fl), BH, S, L, d, d ** -0.5, stream(dev))
    return torch.bmm(ds_fl, k), dk_fl, dv_fl


def math_fwd():
    pp = ops.attention_probs(q, k, d ** -0.5)
    return torch.bmm(pp, v)


def math_bwd():
    D = (dout * out).sum(-1)
    call("skp_attn_bwd_kv", ptr(p), ptr(dout), ptr(q), ptr(v), ptr(D), ptr(ds_new), ptr(dv_), ptr(dk_),
         BH, S, L, d, d ** -0.5, stream(dev))
    return torch.bmm(ds_new, k), dk_, dv_


print(f"train fwd: math {timed(math_fwd):.3f} ms  flash {timed(flash_fwd):.3f} ms | "
      f"bwd: math (saved P) {timed(math_bwd):.3f} ms  flash (rebuilt P) {timed(flash_bwd):.3f} ms")
flash_fwd()
a, b = math_bwd(), flash_bwd()
print("flash vs math rel diff dq/dk/dv", [((x - y).abs().max() / x.abs().max()).item() for x, y in zip(a, b)],
      "out", ((o_fl - out).abs().max() / out.abs().max()).item())
