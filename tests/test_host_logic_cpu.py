"""Host-side logic of the UNet-side fusions that needs no GPU: the stacked-projection autograd node
(ops.QKVProjection: one GEMM against [Wq; Wk; Wv], input gradients accumulated into one buffer,
unused outputs skipped) and the lifetime rule of a convolution's GroupNorm statistics partials
(ops._gn_parts_of: dropped once the tensor is written in place).  The HIP paths are in
tests/test_gpu_heads.py and tests/test_gpu_gn_epi.py."""
import torch

from stablekeypoints_amd import ops


def test_qkv_projection_node_matches_separate_projections():
    g = torch.Generator().manual_seed(0)
    x0 = torch.randn(2, 7, 12, generator=g, dtype=torch.float64)
    ws = [torch.randn(8, 12, generator=g, dtype=torch.float64) for _ in range(3)]
    gs = [torch.randn(2, 7, 8, generator=g, dtype=torch.float64) for _ in range(3)]
    w3 = ops._qkv_weight(*ws)
    assert w3 is ops._qkv_weight(*ws)                      # built once per weight set
    x = x0.clone().requires_grad_(True)
    q, k, v = ops.QKVProjection.apply(x, w3, 8)
    assert q.shape == k.shape == v.shape == (2, 7, 8)
    (q * gs[0] + k * gs[1] + v * gs[2]).sum().backward()
    xr = x0.clone().requires_grad_(True)
    outs = [xr @ w.t() for w in ws]
    sum((o * gg).sum() for o, gg in zip(outs, gs)).backward()
    for a, b in zip((q, k, v), outs):
        assert torch.allclose(a, b, rtol=1e-12, atol=1e-12)
    assert torch.allclose(x.grad, xr.grad, rtol=1e-12, atol=1e-12)


def test_qkv_projection_unused_output_and_two_way_split():
    g = torch.Generator().manual_seed(1)
    x0 = torch.randn(3, 5, 6, generator=g, dtype=torch.float64)
    wk, wv = (torch.randn(4, 6, generator=g, dtype=torch.float64) for _ in range(2))
    x = x0.clone().requires_grad_(True)
    k, v = ops.QKVProjection.apply(x, ops._qkv_weight(wk, wv), 4)
    (v * 2.0).sum().backward()                              # k unused: its gradient is skipped
    ref = (torch.full((3, 5, 4), 2.0, dtype=torch.float64) @ wv)
    assert torch.allclose(x.grad, ref, rtol=1e-12, atol=1e-12)


def test_qkv_weight_rebuilt_when_a_weight_changes():
    ws = [torch.randn(4, 4) for _ in range(3)]
    w3 = ops._qkv_weight(*ws)
    ws[1].add_(1.0)                                         # version bump
    w3b = ops._qkv_weight(*ws)
    assert w3b is not w3 and torch.equal(w3b[4:8], ws[1])


def test_gn_partials_dropped_after_in_place_write():
    y = torch.zeros(2, 4, 8, 8)
    part = torch.zeros(2, 4, 1, 2)
    y._skp_gn = (y._version, part, 1)
    got = ops._gn_parts_of(y)
    assert got is not None and got[0] is part and got[1] == 1
    y.mul_(2.0)
    assert ops._gn_parts_of(y) is None
    assert ops._gn_parts_of(torch.zeros(3)) is None          # a tensor no convolution produced
