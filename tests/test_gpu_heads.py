"""In-place head GEMMs of the captured layers (ops.CaptureLogitsHeads / ops.AttnPVHeads on
skp_bgemm_f32_2b) against the reference's head-permuted form (ptp_utils.py:481-541:
reshape_heads_to_batch_dim, einsum q kᵀ·scale, softmax, bmm with v, reshape_batch_dim_to_heads) in
fp64 torch: forward values and the gradients of q, the shared k and v projections, at the SD-1.5 /
SDXL capture shapes.  Tolerance: 1e-5 of each tensor's maximum (fp32 MFMA sums vs fp64)."""
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


@pytest.mark.parametrize("B,S,N,H,d", [(8, 256, 500, 8, 160), (8, 1024, 500, 8, 80), (2, 1024, 500, 20, 64),
                                       (3, 64, 12, 4, 8)])
def test_heads_gemms_match_the_permuted_reference(B, S, N, H, d):
    from stablekeypoints_amd import ops
    g = torch.Generator(device=DEV).manual_seed(S + N + H)
    C = H * d
    q0 = torch.randn(B, S, C, device=DEV, generator=g)
    k0 = torch.randn(1, N, C, device=DEV, generator=g)
    v0 = torch.randn(1, N, C, device=DEV, generator=g)
    wz = torch.randn(B * H, S, N, device=DEV, generator=g)
    wo = torch.randn(B, S, C, device=DEV, generator=g)
    scale = d ** -0.5
    q, k, v = (t.clone().requires_grad_(True) for t in (q0, k0, v0))
    z = ops.capture_logits_heads(q, k, H, scale)
    out = ops.attn_pv_heads(z.softmax(dim=-1), v, H)
    ((z * wz).sum() + (out * wo).sum()).backward()
    qr, kr, vr = (t.double().clone().requires_grad_(True) for t in (q0, k0, v0))
    zr = torch.einsum("bid,bjd->bij", _heads(qr, H), _heads(kr.expand(B, -1, -1), H)) * scale
    o = torch.bmm(zr.softmax(dim=-1), _heads(vr.expand(B, -1, -1), H))
    outr = o.reshape(B, H, S, d).permute(0, 2, 1, 3).reshape(B, S, C)
    ((zr * wz.double()).sum() + (outr * wo.double()).sum()).backward()
    for name, a, b in (("z", z, zr), ("out", out, outr), ("dq", q.grad, qr.grad), ("dk", k.grad, kr.grad),
                       ("dv", v.grad, vr.grad)):
        err = float((a.double() - b).abs().max() / b.abs().max())
        assert err < 1e-5, (name, err)


@pytest.mark.parametrize("B,S,C", [(8, 4096, 320), (8, 256, 1280), (2, 64, 96)])
def test_qkv_projection_matches_three_linears(B, S, C):
    """ops.QKVProjection (one GEMM against [Wq; Wk; Wv], input gradients accumulated by the GEMM)
    against diffusers' three bias-free to_q / to_k / to_v Linears with autograd's gradient sum."""
    from stablekeypoints_amd import ops
    g = torch.Generator(device=DEV).manual_seed(B * S + C)
    x0 = torch.randn(B, S, C, device=DEV, generator=g)
    ws = [torch.randn(C, C, device=DEV, generator=g) / C ** 0.5 for _ in range(3)]
    gs = [torch.randn(B, S, C, device=DEV, generator=g) for _ in range(3)]
    x = x0.clone().requires_grad_(True)
    q, k, v = ops.qkv_projection(x, *ws)
    (q * gs[0] + k * gs[1] + v * gs[2]).sum().backward()
    xr = x0.double().requires_grad_(True)
    outs = [xr @ w.double().t() for w in ws]
    sum((o * gg.double()).sum() for o, gg in zip(outs, gs)).backward()
    for a, b in zip((q, k, v), outs):
        assert float((a.double() - b).abs().max() / b.abs().max()) < 1e-5
    assert float((x.grad.double() - xr.grad).abs().max() / xr.grad.abs().max()) < 1e-5
    # only some of the three used: the missing gradients are skipped
    x2 = x0.clone().requires_grad_(True)
    q2, _, v2 = ops.qkv_projection(x2, *ws)
    (q2 * gs[0] + v2 * gs[2]).sum().backward()
    ref = gs[0].double() @ ws[0].double() + gs[2].double() @ ws[2].double()
    assert float((x2.grad.double() - ref).abs().max() / ref.abs().max()) < 1e-5
