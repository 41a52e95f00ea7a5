"""The SDXL-era store API (unsupervised_keypoints/sdxl_monkey_patch.py, reference
sdxl_monkey_patch.py:8-214) fed by this package's SDXL UNet on the GPU: every attention module under
down / mid / up goes through the controller, the store keeps the ≤ 32² layers of the conditional
half per place, and the patched UNet's output equals the unpatched one (the store hands the
probabilities back unchanged).  The class itself is pinned bit-for-bit against the reference's on
the CPU (tests/test_store_cpu.py)."""
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def _sample(o):
    if isinstance(o, dict):
        return o["sample"]
    return o[0] if isinstance(o, tuple) else getattr(o, "sample", o)


def test_sdxl_store_filled_by_tiny_sdxl_pass():
    from stablekeypoints_amd.optimize_token import load_ldm
    from stablekeypoints_amd.sd import SDXLUNet
    from unsupervised_keypoints import sdxl_monkey_patch as sm
    ldm, _, _ = load_ldm(DEV, "tiny-xl", feature_upsample_res=32, early_exit=False)
    unet = ldm.unet
    assert isinstance(unet, SDXLUNet)
    g = torch.Generator().manual_seed(3)
    lat = torch.randn(1, 4, 32, 32, generator=g).to(DEV).repeat(2, 1, 1, 1)        # (uncond, cond) halves
    ctx = torch.randn(2, 12, unet.cross_attention_dim, generator=g).to(DEV)
    with torch.no_grad():
        ref = _sample(unet(lat, 10, ctx))
    n_mod = sum(1 for name, net in unet.named_children() if any(p in name for p in ("down", "mid", "up"))
                for m in net.modules() if m.__class__.__name__ == "CrossAttention")
    store = sm.AttentionStore()
    count = sm.register_attention_control(ldm, store)
    assert count == n_mod and store.num_att_layers == n_mod and count > 0
    with torch.no_grad():
        out = _sample(unet(lat, 10, ctx))
    # one UNet pass = one diffusion step: between_steps moved the step's lists into attention_store
    assert store.cur_step == 1 and store.cur_att_layer == 0
    assert set(store.attention_store) == set(sm.AttentionStore.get_empty_store())
    kept = sum(len(v) for v in store.attention_store.values())
    assert kept > 0
    for key, maps in store.attention_store.items():
        for m in maps:
            assert m.shape[1] <= 32 ** 2
            assert torch.allclose(m.sum(-1), torch.ones_like(m.sum(-1)), atol=1e-5)   # probabilities
    assert store.attention_store["mid_cross"] and store.attention_store["up_cross"]
    avg = store.get_average_attention()
    for key in avg:
        for a, m in zip(avg[key], store.attention_store[key]):
            assert torch.equal(a, m / 1)
    err = ((out - ref).abs().max() / ref.abs().max()).item()
    print(f"\nSDXL store: {count} attention modules patched, {kept} maps kept; output vs unpatched rel-max {err:.1e}")
    assert err < 1e-4, err
