"""The norm-with-passthrough nodes (ops.LayerNormRes / ops.GroupNormActRes): the gradient of x's
second consumer (the residual add of diffusers' BasicTransformerBlock / ResnetBlock2D /
Transformer2DModel, the UNet the reference's capture rides on, ptp_utils.py:481-506) is added
inside the LayerNorm / GroupNorm backward kernel (skp_layernorm_bwd_add / skp_groupnorm_bwd_add).
Against the same graph built from the plain nodes (LayerNormFn / GroupNormAct) with the residual's
gradient summed by autograd: outputs and input gradients bit-identical (one fp32 add either way)."""
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")


@pytest.mark.parametrize("rows,C", [(32768, 320), (8192, 640), (2048, 1280), (4096, 96)])
def test_layer_norm_res_equals_plain_plus_autograd_sum(rows, C):
    from stablekeypoints_amd import ops
    g = torch.Generator(device=DEV).manual_seed(rows + C)
    x0 = torch.randn(8, rows // 8, C, device=DEV, generator=g) * 3 + 1
    w = torch.randn(C, device=DEV, generator=g)
    b = torch.randn(C, device=DEV, generator=g)
    wa = torch.randn(C, C, device=DEV, generator=g) / C ** 0.5
    go = torch.randn(8, rows // 8, C, device=DEV, generator=g)
    outs = []
    for fused in (True, False):
        x = x0.clone().requires_grad_(True)
        h = x * 1.0                                   # an interior node, as in the UNet
        if fused:
            y, hp = ops.layer_norm_res(h, w, b, 1e-5)
        else:
            y, hp = ops.LayerNormFn.apply(h, w, b, 1e-5), h
        out = (y @ wa) + hp                           # attn(norm(h)) + h
        (out * go).sum().backward()
        outs.append((out.detach(), x.grad))
    assert torch.equal(outs[0][0], outs[1][0])
    assert torch.equal(outs[0][1], outs[1][1])


@pytest.mark.parametrize("shape,groups,act,shortcut", [((8, 320, 64, 64), 32, True, False),
                                                        ((8, 640, 32, 32), 32, True, True),
                                                        ((8, 1280, 16, 16), 32, False, False),
                                                        ((2, 96, 10, 10), 32, True, False)])
def test_group_norm_act_res_equals_plain_plus_autograd_sum(shape, groups, act, shortcut):
    from stablekeypoints_amd import ops
    g = torch.Generator(device=DEV).manual_seed(sum(shape))
    C = shape[1]
    x0 = torch.randn(*shape, device=DEV, generator=g) * 2 + 0.5
    gamma = torch.randn(C, device=DEV, generator=g)
    beta = torch.randn(C, device=DEV, generator=g)
    ws = torch.randn(C, C, device=DEV, generator=g) / C ** 0.5
    go = torch.randn(*shape, device=DEV, generator=g)
    outs = []
    for fused in (True, False):
        x = x0.clone().requires_grad_(True)
        h = x * 1.0
        if fused:
            y, hp = ops.group_norm_act_res(h, gamma, beta, groups, 1e-5, act)
        else:
            y, hp = ops.GroupNormAct.apply(h, gamma, beta, groups, 1e-5, act, None), h
        res = torch.einsum("oc,bchw->bohw", ws, hp) if shortcut else hp   # 1×1 shortcut or identity
        out = y * 0.5 + res
        (out * go).sum().backward()
        outs.append((out.detach(), x.grad))
    assert torch.equal(outs[0][0], outs[1][0])
    assert torch.equal(outs[0][1], outs[1][1])
