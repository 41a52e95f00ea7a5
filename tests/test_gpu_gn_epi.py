"""GroupNorm statistics from the producing convolution's epilogue (skp_conv3x3_wino2_gn →
skp_groupnorm_fwd_part): the UNet / VAE resnet's conv → GroupNorm(+SiLU) pair (diffusers resnet.py, the
network the reference's capture rides on, ptp_utils.py:481-506).

Checks: the per-segment (mean, M2) partials (r05: accumulated around a pivot inside the segment,
then Chan's combination) against fp64 segment means (1e-5 of the segment's mean |y|) and centred
second moments (1e-5 relative, plus a floor); the GroupNorm output against fp64 torch GroupNorm of the same conv output
(2e-5 of max |y|, the same bound the plain statistics pass meets) and against the statistics-pass
path (ops.GN_EPI = False); an in-place write to the conv output drops the partials."""
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")


def _gn_ref(x, shift, gamma, beta, G, eps, act):
    x = x.double()
    if shift is not None:
        x = x + shift.double()[:, :, None, None]
    y = torch.nn.functional.group_norm(x, G, gamma.double(), beta.double(), eps)
    return torch.nn.functional.silu(y) if act else y


@pytest.mark.parametrize("B,C,K,H,W,res,shift,act", [(8, 320, 320, 64, 64, False, True, True),
                                                      (2, 128, 128, 256, 256, True, False, True),
                                                      (2, 256, 512, 64, 96, False, False, False),
                                                      (4, 320, 320, 64, 64, True, True, True)])
def test_conv_epilogue_groupnorm_statistics(monkeypatch, B, C, K, H, W, res, shift, act):
    from stablekeypoints_amd import ops
    g = torch.Generator(device=DEV).manual_seed(B * C + K + H)
    x = torch.randn(B, C, H, W, device=DEV, generator=g)
    w = torch.randn(K, C, 3, 3, device=DEV, generator=g) / (3 * C ** 0.5)
    bias = torch.randn(K, device=DEV, generator=g) * 0.5 + 1.0
    r = torch.randn(B, K, H, W, device=DEV, generator=g) if res else None
    sh = torch.randn(B, K, device=DEV, generator=g) if shift else None
    gamma = torch.randn(K, device=DEV, generator=g)
    beta = torch.randn(K, device=DEV, generator=g)
    assert ops._wino_plan(B, C, K, H, W)[:2] == (True, 1), "shape must take the one-split Winograd kernel"
    y = ops.conv3x3(x, w, bias, r)
    parts = ops._gn_parts_of(y)
    assert parts is not None, "the convolution left no statistics partials"
    gp, nseg = parts
    assert nseg == (H // 16) * (W // 32)
    _check_parts(gp, y.double().reshape(B, K, H // 16, 16, W // 32, 32).permute(0, 1, 2, 4, 3, 5)
                 .reshape(B, K, nseg, 512))

    out = ops.group_norm_act(y, gamma, beta, 32, 1e-5, act, sh)
    ref = _gn_ref(y, sh, gamma, beta, 32, 1e-5, act)
    scale = float(ref.abs().max())
    assert float((out.double() - ref).abs().max()) / scale < 2e-5
    monkeypatch.setattr(ops, "GN_EPI", False)
    plain = ops.group_norm_act(y, gamma, beta, 32, 1e-5, act, sh)
    assert float((out - plain).abs().max()) / scale < 2e-5
    monkeypatch.setattr(ops, "GN_EPI", True)

    y.add_(1.0)                                      # stale partials must not be used
    assert ops._gn_parts_of(y) is None
    out2 = ops.group_norm_act(y, gamma, beta, 32, 1e-5, act, sh)
    ref2 = _gn_ref(y, sh, gamma, beta, 32, 1e-5, act)
    assert float((out2.double() - ref2).abs().max()) / float(ref2.abs().max()) < 2e-5


def _check_parts(gp, vals):
    """gp (B, K, nseg) float2 (mean, M2) vs fp64 over vals (B, K, nseg, n)."""
    mean = vals.mean(-1)
    m2 = ((vals - mean[..., None]) ** 2).sum(-1)
    a1 = vals.abs().mean(-1)
    assert float(((gp[..., 0].double() - mean).abs() / a1).max()) < 1e-5
    assert float(((gp[..., 1].double() - m2).abs() / (m2 + 1e-6 * a1 * a1 * vals.shape[-1])).max()) < 1e-5


@pytest.mark.parametrize("B,C,K,H,W,offset", [(2, 128, 128, 256, 256, 50.0), (8, 320, 320, 64, 64, 400.0)])
def test_conv_epilogue_groupnorm_large_offset(B, C, K, H, W, offset):
    """A channel mean far from 0 relative to its spread (bias ≈ 50, std ≈ 1, plus a time
    -embedding shift): the epilogue statistics (pivoted (mean, M2), Chan's combination in fp64) give
    the GroupNorm output within 2e-5 of fp64 torch; E[x²] − mean² from fp32 (Σx, Σx²), the r04 form,
    lost the variance here."""
    from stablekeypoints_amd import ops
    assert ops._wino_plan(B, C, K, H, W)[:2] == (True, 1), "shape must take the one-split Winograd kernel"
    g = torch.Generator(device=DEV).manual_seed(int(offset))
    x = torch.randn(B, C, H, W, device=DEV, generator=g)
    w = torch.randn(K, C, 3, 3, device=DEV, generator=g) / (3 * C ** 0.5)   # output std ≈ 1
    bias = offset + torch.randn(K, device=DEV, generator=g) * 0.1
    sh = torch.randn(B, K, device=DEV, generator=g) * (offset / 5)
    gamma = torch.randn(K, device=DEV, generator=g)
    beta = torch.randn(K, device=DEV, generator=g)
    y = ops.conv3x3(x, w, bias)
    parts = ops._gn_parts_of(y)
    assert parts is not None
    gp, nseg = parts
    _check_parts(gp, y.double().reshape(B, K, H // 16, 16, W // 32, 32).permute(0, 1, 2, 4, 3, 5)
                 .reshape(B, K, nseg, 512))
    out = ops.group_norm_act(y, gamma, beta, 32, 1e-5, True, sh)
    ref = _gn_ref(y, sh, gamma, beta, 32, 1e-5, True)
    err = float((out.double() - ref).abs().max()) / float(ref.abs().max())
    print(f"\nGroupNorm from epilogue statistics at offset {offset}: rel-max {err:.1e}")
    assert err < 2e-5, err


def test_resnet_block_with_epilogue_statistics_matches_plain(monkeypatch):
    """A fused ResnetBlock2D forward + input gradient with and without the epilogue statistics."""
    from stablekeypoints_amd import ops
    from stablekeypoints_amd.sd.unet import ResnetBlock2D
    torch.manual_seed(0)
    blk = ResnetBlock2D(320, 320, temb_channels=1280).to(DEV).eval().requires_grad_(False)
    g = torch.Generator(device=DEV).manual_seed(3)
    x0 = torch.randn(8, 320, 64, 64, device=DEV, generator=g)
    temb = torch.randn(8, 1280, device=DEV, generator=g)
    go = torch.randn(8, 320, 64, 64, device=DEV, generator=g)
    outs = []
    for on in (True, False):
        monkeypatch.setattr(ops, "GN_EPI", on)
        x = ops.conv3x3(x0, blk.conv2.weight, blk.conv2.bias).requires_grad_(True)   # a leaf
        assert (ops._gn_parts_of(x) is not None) == on
        y = blk(x, temb)
        (y * go).sum().backward()
        outs.append((y.detach(), x.grad))
    for a, b in zip(outs[0], outs[1]):
        assert float((a - b).abs().max()) / float(b.abs().max()) < 1e-4


@pytest.mark.parametrize("B,C,K,H,W,res", [(8, 640, 640, 32, 32, True), (8, 1280, 1280, 16, 16, False),
                                           (4, 256, 256, 16, 32, False), (2, 256, 320, 32, 64, True)])
def test_wino_gemm_groupnorm_statistics(monkeypatch, B, C, K, H, W, res):
    """The Winograd-GEMM form (skp_wino_out_transform_kt): the same partials per segment of
    min(P, 64) tiles, output within 3e-5 of the fp64 convolution."""
    from stablekeypoints_amd import ops
    g = torch.Generator(device=DEV).manual_seed(B + C + K + H + W)
    x = torch.randn(B, C, H, W, device=DEV, generator=g)
    w = torch.randn(K, C, 3, 3, device=DEV, generator=g) / (3 * C ** 0.5)
    bias = torch.randn(K, device=DEV, generator=g)
    r = torch.randn(B, K, H, W, device=DEV, generator=g) if res else None
    monkeypatch.setattr(ops, "WINO_GEMM_MAX_HW", max(ops.WINO_GEMM_MAX_HW, H * W))   # 2 segments per plane
    assert ops._wino_gemm_ok(B, C, K, H, W)
    y = ops.conv3x3(x, w, bias, r)
    gp, nseg = ops._gn_parts_of(y)
    th, tw = H // 4, W // 4
    P = th * tw
    seg = min(P, 64)
    assert nseg == P // seg
    tiles = y.double().reshape(B, K, th, 4, tw, 4).permute(0, 1, 2, 4, 3, 5).reshape(B, K, P, 16)
    _check_parts(gp, tiles.reshape(B, K, nseg, seg * 16))
    ref = torch.nn.functional.conv2d(x.double(), w.double(), bias.double(), padding=1)
    if r is not None:
        ref = ref + r.double()
    assert float((y.double() - ref).abs().max()) <= 3e-5 * float(ref.abs().max())
