"""skp_conv3x3_wino (Winograd F(4×4, 3×3) on the fp32 matrix cores) vs torch fp64.

The VAE encoder and UNet 3×3 convolutions run through ops.conv3x3.  Tolerance: the max
error relative to the output's max magnitude stays below 3e-5 (a direct fp32 sum of the same
length sits near 1e-6; F(4×4) with the points (0, ±1, 1/2, -2) measured ≈3× that on CPU, the
bound leaves room for accumulation order).  Input gradients are checked the same way.
"""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

DEV = "cuda:0"


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")


@pytest.fixture
def all_shapes(monkeypatch):
    from stablekeypoints_amd import ops
    monkeypatch.setattr(ops, "WINO_MIN_WORKGROUPS", 1)
    monkeypatch.setattr(ops, "WINO_GEMM_MAX_HW", 0)   # these tests cover the fused kernels
    return ops


def _rel(a, b):
    return ((a.double() - b).abs().max() / b.abs().max()).item()


@pytest.mark.parametrize("B,C,K,H,W", [(2, 64, 64, 32, 32), (2, 4, 32, 20, 20), (1, 32, 96, 12, 28),
                                       (3, 128, 64, 16, 8), (1, 512, 64, 8, 8), (2, 36, 32, 4, 4),
                                       (1, 8, 32, 32, 32), (2, 12, 64, 64, 96), (1, 40, 32, 96, 32),
                                       (3, 4, 32, 32, 64), (4, 8, 32, 16, 16), (8, 36, 64, 16, 16),
                                       # region-kernel stage counts C/4 of 5, 7 and 11: every tail of
                                       # its 6-step unrolled ring (zero-length raw loads past the end)
                                       (1, 20, 32, 32, 32), (2, 28, 32, 32, 64), (4, 44, 32, 16, 16)])
@pytest.mark.parametrize("bias,res", [(False, False), (True, False), (True, True)])
def test_conv3x3_forward_vs_fp64(all_shapes, B, C, K, H, W, bias, res):
    ops = all_shapes
    g = torch.Generator().manual_seed(B * 1000 + C + K + H)
    x = torch.randn(B, C, H, W, generator=g)
    w = torch.randn(K, C, 3, 3, generator=g) / (3 * C ** 0.5)
    b = torch.randn(K, generator=g) if bias else None
    r = torch.randn(B, K, H, W, generator=g) if res else None
    y = ops.conv3x3(x.to(DEV), w.to(DEV), None if b is None else b.to(DEV), None if r is None else r.to(DEV))
    ref = F.conv2d(x.double(), w.double(), None if b is None else b.double(), 1, 1)
    if r is not None:
        ref = ref + r.double()
    assert y.shape == ref.shape
    assert _rel(y.cpu(), ref) < 3e-5


@pytest.mark.parametrize("B,C,K,H,W", [(2, 64, 32, 16, 16), (1, 32, 64, 12, 20), (2, 320, 320, 8, 8),
                                       (2, 64, 32, 32, 64), (1, 96, 64, 64, 32), (4, 64, 96, 16, 16)])
def test_conv3x3_input_gradient_vs_fp64(all_shapes, B, C, K, H, W):
    ops = all_shapes
    g = torch.Generator().manual_seed(K + H)
    x = torch.randn(B, C, H, W, generator=g)
    w = torch.randn(K, C, 3, 3, generator=g) / (3 * C ** 0.5)
    r = torch.randn(B, K, H, W, generator=g)
    dy = torch.randn(B, K, H, W, generator=g)
    xd, rd = x.to(DEV).requires_grad_(True), r.to(DEV).requires_grad_(True)
    y = ops.conv3x3(xd, w.to(DEV), None, rd)
    (y * dy.to(DEV)).sum().backward()
    x64 = x.double().requires_grad_(True)
    (F.conv2d(x64, w.double(), None, 1, 1) * dy.double()).sum().backward()
    assert _rel(xd.grad.cpu(), x64.grad) < 3e-5
    assert torch.equal(rd.grad.cpu(), dy)


def test_conv3x3_vae_shape_and_weight_cache(all_shapes):
    """A full-size VAE layer (128 channels at 512², batch 1) and the transformed-weight cache:
    an in-place weight update invalidates it."""
    ops = all_shapes
    g = torch.Generator(device=DEV).manual_seed(3)
    x = torch.randn(1, 128, 512, 512, device=DEV, generator=g)
    w = torch.randn(128, 128, 3, 3, device=DEV, generator=g) / 34
    b = torch.randn(128, device=DEV, generator=g)
    y = ops.conv3x3(x, w, b)
    ref = F.conv2d(x.double(), w.double(), b.double(), 1, 1)
    assert _rel(y, ref) < 3e-5
    with torch.no_grad():
        w.mul_(-2.0)
    y2 = ops.conv3x3(x, w, b)
    ref2 = F.conv2d(x.double(), w.double(), b.double(), 1, 1)
    assert _rel(y2, ref2) < 3e-5


@pytest.mark.parametrize("H,W", [(32, 32), (64, 96), (16, 16)])
def test_conv3x3_v2_zero_padding_at_every_edge(all_shapes, H, W):
    """skp_conv3x3_wino2 zero-pads by loading out-of-range rows / 16-B chunks as zeros: a
    constant input must give, at every border pixel and corner, the partial 3×3 sum of the
    in-image taps only (exactly, the weights being small integers)."""
    ops = all_shapes
    assert ops._wino_v2(H, W, 4)
    C, K = 4, 32
    x = torch.ones(4, C, H, W, device=DEV)
    w = torch.randint(-2, 3, (K, C, 3, 3), generator=torch.Generator().manual_seed(5)).float()
    y = ops.conv3x3(x, w.to(DEV))
    ref = F.conv2d(x.cpu().double(), w.double(), None, 1, 1)
    assert (y.cpu().double() - ref).abs().max().item() < 1e-4


@pytest.mark.parametrize("B,HW", [(2, 64), (8, 16)])
def test_conv3x3_v1_v2_agree(all_shapes, monkeypatch, B, HW):
    """The two Winograd kernels compute the same convolution (same transform points; only the
    summation order differs); both block geometries of the region kernel."""
    ops = all_shapes
    g = torch.Generator(device=DEV).manual_seed(9)
    x = torch.randn(B, 64, HW, HW, device=DEV, generator=g)
    w = torch.randn(64, 64, 3, 3, device=DEV, generator=g) / 24
    y2 = ops.conv3x3(x, w)
    monkeypatch.setattr(ops, "WINO_KERNEL", "v1")
    y1 = ops.conv3x3(x, w)
    assert (y1 - y2).abs().max().item() < 1e-5 * y1.abs().max().item()


@pytest.mark.parametrize("B,C,K,H,W", [(2, 256, 64, 16, 16), (1, 384, 32, 32, 32), (2, 512, 64, 8, 8),
                                       (4, 512, 64, 16, 16)])
def test_conv3x3_split_k_vs_fp64_and_unsplit(all_shapes, monkeypatch, B, C, K, H, W):
    """Split-K (input channels over several workgroup sets + one reduction pass with the bias
    and the residual) equals fp64 and the unsplit kernel; the forward and the input gradient."""
    ops = all_shapes
    assert ops._wino_plan(B, C, K, H, W)[1] > 1 and ops._wino_plan(B, K, C, H, W)[1] >= 1
    g = torch.Generator().manual_seed(C + H)
    x = torch.randn(B, C, H, W, generator=g)
    w = torch.randn(K, C, 3, 3, generator=g) / (3 * C ** 0.5)
    b = torch.randn(K, generator=g)
    r = torch.randn(B, K, H, W, generator=g)
    dy = torch.randn(B, K, H, W, generator=g)
    outs = []
    for split in (True, False):
        monkeypatch.setattr(ops, "WINO_SPLIT", split)
        xd = x.to(DEV).requires_grad_(True)
        y = ops.conv3x3(xd, w.to(DEV), b.to(DEV), r.to(DEV))
        (y * dy.to(DEV)).sum().backward()
        outs.append((y.detach().cpu(), xd.grad.cpu()))
    x64 = x.double().requires_grad_(True)
    ref = F.conv2d(x64, w.double(), b.double(), 1, 1) + r.double()
    (ref * dy.double()).sum().backward()
    for y, dx in outs:
        assert _rel(y, ref.detach()) < 3e-5
        assert _rel(dx, x64.grad) < 3e-5
    assert (outs[0][0] - outs[1][0]).abs().max().item() < 1e-5 * outs[1][0].abs().max().item()


@pytest.mark.parametrize("B,C,K,H,W", [(8, 256, 128, 8, 8), (2, 128, 64, 8, 8), (3, 64, 192, 4, 12),
                                       (8, 1280, 1280, 8, 8), (1, 96, 64, 4, 4)])
def test_conv3x3_wide_blocks_vs_fp64(all_shapes, B, C, K, H, W):
    """Grids of at most 32 tiles with K a multiple of 64 run as 32-tile × 64-channel workgroups
    (skp_conv3x3_wino's wide blocks, the UNet's 8² layers): forward with bias + residual and the
    input gradient (wide too when C is a multiple of 64) vs fp64, split-K included."""
    ops = all_shapes
    assert B * (H // 4) * (W // 4) <= 32 and K % 64 == 0
    g = torch.Generator().manual_seed(C * 3 + K)
    x = torch.randn(B, C, H, W, generator=g)
    w = torch.randn(K, C, 3, 3, generator=g) / (3 * C ** 0.5)
    b = torch.randn(K, generator=g)
    r = torch.randn(B, K, H, W, generator=g)
    dy = torch.randn(B, K, H, W, generator=g)
    xd = x.to(DEV).requires_grad_(True)
    y = ops.conv3x3(xd, w.to(DEV), b.to(DEV), r.to(DEV))
    (y * dy.to(DEV)).sum().backward()
    x64 = x.double().requires_grad_(True)
    ref = F.conv2d(x64, w.double(), b.double(), 1, 1) + r.double()
    (ref * dy.double()).sum().backward()
    assert _rel(y.detach().cpu(), ref.detach()) < 3e-5
    assert _rel(xd.grad.cpu(), x64.grad) < 3e-5


def test_conv3x3_batch_above_2gib_runs_in_chunks(all_shapes):
    """An input above 2 GiB (the kernels' 32-bit buffer offsets; the SDXL VAE at 1024², batch 8)
    runs as batch chunks: same result as MIOpen (fp32) over the whole batch, bias and residual
    included."""
    ops = all_shapes
    g = torch.Generator(device=DEV).manual_seed(4)
    x = torch.randn(5, 128, 1024, 1024, device=DEV, generator=g)
    assert x.numel() * 4 > 2 ** 31
    w = torch.randn(128, 128, 3, 3, device=DEV, generator=g) / 34
    b = torch.randn(128, device=DEV, generator=g)
    r = torch.randn_like(x)
    y = ops.conv3x3(x, w, b, r)
    ref = F.conv2d(x, w, b, 1, 1) + r
    assert (y - ref).abs().max().item() < 3e-5 * ref.abs().max().item()


def test_conv3x3_falls_back_to_miopen_for_ineligible_shapes():
    """conv_out (8 output channels) goes to MIOpen, not the Winograd kernel."""
    from stablekeypoints_amd import ops
    x = torch.randn(1, 32, 16, 16, device=DEV)
    w = torch.randn(8, 32, 3, 3, device=DEV)
    assert not ops.wino_eligible(1, 32, 8, 16, 16, min_workgroups=1)
    assert torch.allclose(ops.conv3x3(x, w), F.conv2d(x, w, None, 1, 1), atol=1e-4)


@pytest.mark.parametrize("C", [3, 1, 6])
def test_conv3x3_input_layer_channels_zero_padded(all_shapes, C):
    """conv_in (RGB: 3 channels; latents: 4): channels padded with zeros to a multiple of 4 run on
    the Winograd kernel, forward and input gradient vs fp64, bias included."""
    ops = all_shapes
    g = torch.Generator().manual_seed(C)
    x = torch.randn(4, C, 32, 32, generator=g)
    w = torch.randn(64, C, 3, 3, generator=g) / 3
    b = torch.randn(64, generator=g)
    dy = torch.randn(4, 64, 32, 32, generator=g)
    xd = x.to(DEV).requires_grad_(True)
    y = ops.conv3x3(xd, w.to(DEV), b.to(DEV))
    (y * dy.to(DEV)).sum().backward()
    x64 = x.double().requires_grad_(True)
    ref = F.conv2d(x64, w.double(), b.double(), 1, 1)
    (ref * dy.double()).sum().backward()
    assert _rel(y.detach().cpu(), ref.detach()) < 3e-5
    assert _rel(xd.grad.cpu(), x64.grad) < 3e-5


def test_sd_models_winograd_vs_miopen(monkeypatch):
    """The tiny SD UNet (forward + context gradient) and VAE encoder with every eligible 3×3
    convolution on the Winograd kernel equal the same models on MIOpen (within 1e-4)."""
    from stablekeypoints_amd import ops
    from stablekeypoints_amd.sd import build_sd15, TINY_CONFIG
    ldm = build_sd15(seed=0, config=TINY_CONFIG, device=DEV)
    gen = torch.Generator(device=DEV).manual_seed(0)
    img = torch.rand(2, 3, 128, 128, device=DEV, generator=gen) * 2 - 1
    lat = torch.randn(2, 4, 16, 16, device=DEV, generator=gen)
    ctx0 = torch.randn(1, 16, 32, device=DEV, generator=gen)
    outs = []
    for thresh in (10 ** 9, 1):
        monkeypatch.setattr(ops, "WINO_MIN_WORKGROUPS", thresh)
        with torch.no_grad():
            z = ldm.vae.encode(img)["latent_dist"].mean
        ctx = ctx0.clone().requires_grad_(True)
        out = ldm.unet(lat, torch.tensor(0, device=DEV).repeat(2), ctx.repeat(2, 1, 1))["sample"]
        out.square().mean().backward()
        outs.append((z, out.detach(), ctx.grad.detach()))
    for a, b in zip(outs[0], outs[1]):
        assert _rel(b, a.double()) < 1e-4


@pytest.mark.parametrize("B,C,K,H,W,bias,nsplit", [(2, 64, 64, 64, 64, True, 0), (1, 32, 96, 32, 96, True, 0),
                                                   (3, 8, 32, 32, 32, False, 0), (2, 128, 64, 64, 32, True, 4),
                                                   (1, 256, 32, 32, 32, True, 8)])
def test_conv3x3_stride2_downsample_vs_fp64(all_shapes, monkeypatch, B, C, K, H, W, bias, nsplit):
    """ops.conv3x3_s2 (skp_conv3x3s2_wino2: the Winograd kernel with the stride-2 epilogue) vs the
    reference's Downsample2D(padding=0) in fp64: F.pad(x, (0, 1, 0, 1)) then conv2d(stride=2);
    with and without bias, unsplit and split-K (the sums reduced by splitk_reduce)."""
    ops = all_shapes
    monkeypatch.setattr(ops, "WINO_S2_MIN_PIXELS", 1)
    if nsplit:
        monkeypatch.setattr(ops, "WINO_NSPLIT_FORCE", nsplit)
    g = torch.Generator().manual_seed(B * 1000 + C + K + H)
    x = torch.randn(B, C, H, W, generator=g)
    w = torch.randn(K, C, 3, 3, generator=g) / (3 * C ** 0.5)
    b = torch.randn(K, generator=g) if bias else None
    ref = F.conv2d(F.pad(x.double(), (0, 1, 0, 1)), w.double(), None if b is None else b.double(), stride=2)
    with torch.no_grad():
        y = ops.conv3x3_s2(x.to(DEV), w.to(DEV), None if b is None else b.to(DEV))
    assert y.shape == ref.shape
    assert _rel(y.cpu(), ref) < 3e-5


def test_vae_downsample_uses_stride2_winograd_and_matches_miopen(monkeypatch):
    """The VAE's Downsample2D takes the stride-2 Winograd path under no_grad and equals the
    F.pad + MIOpen path (the ops.WINO_S2 = False form) at 128 channels, batch 2."""
    from stablekeypoints_amd import ops
    from stablekeypoints_amd.sd.unet import Downsample2D
    torch.manual_seed(0)
    m = Downsample2D(128, padding=0).to(DEV)
    for p in m.parameters():
        p.requires_grad_(False)
    x = torch.randn(2, 128, 512, 384, device=DEV)
    calls = []
    real = ops.conv3x3_s2
    monkeypatch.setattr(ops, "conv3x3_s2", lambda *a: calls.append(1) or real(*a))
    with torch.no_grad():
        y = m(x)
        assert calls, "Downsample2D did not take the stride-2 Winograd path"
        monkeypatch.setattr(ops, "WINO_S2", False)
        y2 = m(x)
    assert y.shape == (2, 128, 256, 192)
    assert ((y - y2).abs().max() / y2.abs().max()).item() < 3e-5


@pytest.mark.parametrize("B,C,K,H,W", [(2, 320, 640, 16, 16), (3, 96, 32, 8, 12), (1, 2560, 1280, 8, 8)])
def test_conv1x1_gemm_vs_fp64(B, C, K, H, W):
    """ops.conv1x1 (one batched GEMM on NCHW, the resnets' shortcut) vs conv2d in fp64: output and
    input gradient."""
    from stablekeypoints_amd import ops
    ops.CONV1X1_GEMM, saved = True, ops.CONV1X1_GEMM
    g = torch.Generator().manual_seed(C + K + H)
    x = torch.randn(B, C, H, W, generator=g)
    w = torch.randn(K, C, 1, 1, generator=g) / C ** 0.5
    dy = torch.randn(B, K, H, W, generator=g)
    x64 = x.double().requires_grad_(True)
    ref = F.conv2d(x64, w.double())
    ref.backward(dy.double())
    xd = x.to(DEV).requires_grad_(True)
    try:
        y = ops.conv1x1(xd, w.to(DEV))
    finally:
        ops.CONV1X1_GEMM = saved
    y.backward(dy.to(DEV))
    assert _rel(y.detach().cpu(), ref.detach()) < 1e-5
    assert _rel(xd.grad.cpu(), x64.grad) < 1e-5


def test_resnet_block_shortcut_gemm_matches_miopen_form(monkeypatch):
    """ResnetBlock2D with a 1×1 shortcut: the fused form (shortcut GEMM, its bias folded into conv2's
    epilogue) equals the MIOpen shortcut form (ops.CONV1X1_GEMM = False), forward and input gradient."""
    from stablekeypoints_amd import ops
    from stablekeypoints_amd.sd.unet import ResnetBlock2D
    torch.manual_seed(1)
    m = ResnetBlock2D(64, 128, temb_channels=256).to(DEV)
    for p in m.parameters():
        p.requires_grad_(False)
    x = torch.randn(4, 64, 32, 32, device=DEV, requires_grad=True)
    temb = torch.randn(4, 256, device=DEV)
    monkeypatch.setattr(ops, "CONV1X1_GEMM", True)
    y = m(x, temb)
    y.square().sum().backward()
    gx = x.grad.clone()
    x.grad = None
    monkeypatch.setattr(ops, "CONV1X1_GEMM", False)
    y2 = m(x, temb)
    y2.square().sum().backward()
    assert ((y - y2).abs().max() / y2.abs().max()).item() < 3e-5
    assert ((gx - x.grad).abs().max() / x.grad.abs().max()).item() < 3e-5


# ----------------------------------------------------------------------------- Winograd as batched GEMMs
@pytest.mark.parametrize("B,C,K,H,W", [(8, 1280, 1280, 16, 16), (8, 2560, 1280, 8, 8), (8, 640, 640, 32, 32),
                                       (3, 256, 320, 12, 20), (1, 320, 256, 4, 4)])
@pytest.mark.parametrize("bias,res", [(False, False), (True, True)])
def test_conv3x3_wino_gemm_vs_fp64(monkeypatch, B, C, K, H, W, bias, res):
    """skp_wino_in_transform → 36 batched GEMMs → skp_wino_out_transform (the UNet's 8²-32²
    layers) vs fp64 conv2d: forward with bias / residual, and the input gradient (the same path on
    the rotated weights), at the fused kernels' 3e-5 bound."""
    from stablekeypoints_amd import ops
    monkeypatch.setattr(ops, "WINO_MIN_WORKGROUPS", 1)
    monkeypatch.setattr(ops, "WINO_GEMM_MAX_HW", 1024)
    assert ops._wino_gemm_ok(B, C, K, H, W) and ops._wino_gemm_ok(B, K, C, H, W)
    g = torch.Generator().manual_seed(B + C + K + H + W)
    x = torch.randn(B, C, H, W, generator=g)
    w = torch.randn(K, C, 3, 3, generator=g) / (3 * C ** 0.5)
    b = torch.randn(K, generator=g) if bias else None
    r = torch.randn(B, K, H, W, generator=g) if res else None
    dy = torch.randn(B, K, H, W, generator=g)
    xd = x.to(DEV).requires_grad_(True)
    y = ops.conv3x3(xd, w.to(DEV), None if b is None else b.to(DEV), None if r is None else r.to(DEV))
    (y * dy.to(DEV)).sum().backward()
    x64 = x.double().requires_grad_(True)
    ref = F.conv2d(x64, w.double(), None if b is None else b.double(), 1, 1)
    if r is not None:
        ref = ref + r.double()
    (ref * dy.double()).sum().backward()
    assert _rel(y.detach().cpu(), ref.detach()) < 3e-5
    assert _rel(xd.grad.cpu(), x64.grad) < 3e-5


def test_conv3x3_wino_gemm_equals_fused_kernel_closely(monkeypatch):
    """The GEMM form and the fused kernel compute the same F(4×4, 3×3) transform: at a UNet 16²
    shape they agree far inside the fp64 bound."""
    from stablekeypoints_amd import ops
    g = torch.Generator().manual_seed(5)
    x = torch.randn(8, 1280, 16, 16, generator=g).to(DEV)
    w = (torch.randn(1280, 1280, 3, 3, generator=g) / (3 * 1280 ** 0.5)).to(DEV)
    monkeypatch.setattr(ops, "WINO_GEMM_MAX_HW", 0)
    y0 = ops.conv3x3(x, w)
    monkeypatch.setattr(ops, "WINO_GEMM_MAX_HW", 1024)
    y1 = ops.conv3x3(x, w)
    assert ((y0 - y1).abs().max() / y0.abs().max()).item() < 2e-5
