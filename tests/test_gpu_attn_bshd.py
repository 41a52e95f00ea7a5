"""Attention on the projections' own (B, S, H·d) layout (ops.attention_heads: skp_attn_fwd_bshd /
skp_attn_bwd_flash_bshd) vs plain fp32 torch on the head-permuted tensors — diffusers 0.8.0's
CrossAttention math path (reshape_heads_to_batch_dim → softmax(q kᵀ·scale) v →
reshape_batch_dim_to_heads; reference ptp_utils.py:481-506 for the layers the capture leaves alone).

Cases: self-attention (L = S), cross-attention with a batch-shared context (the token embedding
expanded over the batch: zero batch stride, ragged key count), head dims 40 and 64, forward and
the gradients of q, k, v.  Tolerance 2e-5 relative to the largest magnitude (fp32 reordering)."""
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")


def _heads(t, H):
    b, s, c = t.shape
    return t.reshape(b, s, H, c // H).permute(0, 2, 1, 3).reshape(b * H, s, c // H)


def _merge(t, H):
    bh, s, d = t.shape
    return t.reshape(bh // H, H, s, d).permute(0, 2, 1, 3).reshape(bh // H, s, d * H)


def _ref(q, k, v, H, scale):
    qh, kh, vh = (_heads(t, H) for t in (q, k, v))
    p = torch.softmax(torch.bmm(qh, kh.transpose(1, 2)) * scale, dim=-1)
    return _merge(torch.bmm(p, vh), H)


def _rel(a, b):
    return float((a - b).abs().max() / b.abs().max().clamp_min(1e-30))


@pytest.mark.parametrize("B,H,S,L,d,shared", [
    (2, 8, 256, 256, 40, False),     # self-attention, the UNet's 64² head dim (kernels called directly)
    (2, 8, 192, 77, 40, True),       # cross-attention, batch-shared context, ragged keys
    (3, 4, 128, 128, 64, False),     # SDXL's head dim
    (2, 5, 64, 500, 64, True),       # 500 tokens (the bench's N), shared
])
def test_attention_heads_fwd_bwd_vs_torch(B, H, S, L, d, shared):
    """The BSHD kernels (FlashAttentionBSHD) for shared and per-image k / v; attention_heads routes
    only the shared case with gradients through them (see ops.attention_heads)."""
    from stablekeypoints_amd import ops
    g = torch.Generator(device=DEV).manual_seed(S + L + d)
    C = H * d
    q = torch.randn(B, S, C, device=DEV, generator=g)
    if shared:
        k1 = torch.randn(1, L, C, device=DEV, generator=g)
        v1 = torch.randn(1, L, C, device=DEV, generator=g)
    else:
        k1 = torch.randn(B, L, C, device=DEV, generator=g)
        v1 = torch.randn(B, L, C, device=DEV, generator=g)
    scale = d ** -0.5
    go = torch.randn(B, S, C, device=DEV, generator=g)

    def run(fn):
        qq, kk, vv = (t.clone().requires_grad_(True) for t in (q, k1, v1))
        ke, ve = (kk.expand(B, L, C), vv.expand(B, L, C)) if shared else (kk, vv)
        out = fn(qq, ke, ve)
        assert out is not None
        (out * go).sum().backward()
        return out.detach(), qq.grad, kk.grad, vv.grad

    got = run(lambda a, b, c: ops.FlashAttentionBSHD.apply(a, b, c, H, scale))
    ref = run(lambda a, b, c: _ref(a, b, c, H, scale))
    for name, x, y in zip(("out", "dq", "dk", "dv"), got, ref):
        assert _rel(x, y) < 2e-5, (name, _rel(x, y))


def test_attention_heads_nograd_and_fallbacks():
    from stablekeypoints_amd import ops
    g = torch.Generator(device=DEV).manual_seed(3)
    B, H, S, d = 2, 8, 128, 80
    q, k, v = (torch.randn(B, S, H * d, device=DEV, generator=g) for _ in range(3))
    with torch.no_grad():
        out = ops.attention_heads(q, k, v, H, d ** -0.5)       # d = 80: no-grad online-softmax form
        assert _rel(out, _ref(q, k, v, H, d ** -0.5)) < 2e-5
        assert ops.attention_heads(q[:, :100], k, v, H, 0.1) is None              # S not a multiple of 64
    qg = q.clone().requires_grad_(True)
    assert ops.attention_heads(qg, k, v, H, 0.1) is None        # d = 80 with grad: the caller's path
    q40, k40 = (torch.randn(B, S, 320, device=DEV, generator=g) for _ in range(2))
    assert ops.attention_heads(q40.requires_grad_(True), k40, k40, 8, 0.1) is None   # self-attention with grad
    assert ops.attention_heads(q40, k40[:1].expand(B, -1, -1), k40[:1].expand(B, -1, -1), 8, 0.1) is not None


def test_unet_cross_attention_module_uses_bshd_and_matches_permuting_path(monkeypatch):
    """CrossAttention.forward through the BSHD path equals the r02 permuting path (ops.ATTN_BSHD = False)."""
    from stablekeypoints_amd import ops
    from stablekeypoints_amd.sd.unet import CrossAttention
    torch.manual_seed(0)
    m = CrossAttention(320, cross_attention_dim=768, heads=8, dim_head=40).to(DEV)
    for p in m.parameters():
        p.requires_grad_(False)
    x = torch.randn(2, 256, 320, device=DEV, requires_grad=True)
    ctx = torch.randn(1, 77, 768, device=DEV, requires_grad=True)
    calls = []
    real = ops.attention_heads
    monkeypatch.setattr(ops, "attention_heads", lambda *a: calls.append(1) or real(*a))
    out = m(x, ctx.expand(2, -1, -1))
    assert calls, "the BSHD path did not run"
    out.square().sum().backward()
    gx, gc = x.grad.clone(), ctx.grad.clone()
    x.grad = None
    ctx.grad = None
    monkeypatch.setattr(ops, "ATTN_BSHD", False)
    out2 = m(x, ctx.expand(2, -1, -1))
    out2.square().sum().backward()
    assert _rel(out, out2) < 2e-5 and _rel(gx, x.grad) < 2e-5 and _rel(gc, ctx.grad) < 2e-5


@pytest.mark.parametrize("B,H,S,L,d", [
    (8, 8, 256, 500, 160),     # the 16² cross-attention layers at the bench shape (d = 160)
    (8, 8, 1024, 500, 80),     # the 32² cross-attention layers (d = 80)
    (3, 8, 64, 77, 160),       # a ragged key count, an odd batch
])
def test_shared_context_head_major_vs_torch(B, H, S, L, d):
    """sd.unet.shared_context_attention (heads outermost, one GEMM per head over all B·S query
    rows against the ONE shared key / value sequence) against the batch-expanded, head-permuted
    plain fp32 form: output and the gradients of q and of the single k / v sequence (the
    expanded form's gradients summed over the batch, as the expand's backward does)."""
    from stablekeypoints_amd.sd import unet
    g = torch.Generator(device="cpu").manual_seed(d + S)
    C = H * d
    scale = d ** -0.5
    q = torch.randn(B, S, C, generator=g).to(DEV).requires_grad_()
    k1 = torch.randn(1, L, C, generator=g).to(DEV).requires_grad_()
    v1 = torch.randn(1, L, C, generator=g).to(DEV).requires_grad_()
    do = torch.randn(B, S, C, generator=g).to(DEV)
    out = unet.shared_context_attention(q, k1, v1, H, scale)
    dq, dk, dv = torch.autograd.grad(out, (q, k1, v1), do)
    qr, kr, vr = (t.detach().clone().requires_grad_() for t in (q, k1, v1))
    ref = _ref(qr, kr.expand(B, -1, -1), vr.expand(B, -1, -1), H, scale)
    rq, rk, rv = torch.autograd.grad(ref, (qr, kr, vr), do)
    assert out.shape == (B, S, C)
    for a, b, name in ((out, ref, "out"), (dq, rq, "dq"), (dk, rk, "dk"), (dv, rv, "dv")):
        assert _rel(a, b) < 2e-5, (name, _rel(a, b))
