"""Frozen SD-1.5 / SDXL UNet, VAE-encoder and DDIM scheduler (PyTorch-ROCm side of the path)."""
from .unet import UNet2DConditionModel, CrossAttention, CaptureComplete
from .sdxl import SDXLUNet, SDXL_CONFIG
from .vae import AutoencoderKL
from .scheduler import DDIMScheduler


class StableDiffusionParts:
    """The three pipeline members the hot path touches: ``unet``, ``vae``, ``scheduler``.

    Stands in for ``StableDiffusionPipeline`` (reference ``optimize_token.py:38-40``);
    the text encoder/tokenizer are frozen and unused by the path, so they are absent.
    """

    def __init__(self, unet, vae, scheduler):
        self.unet = unet
        self.vae = vae
        self.scheduler = scheduler

    def to(self, device):
        self.unet.to(device)
        self.vae.to(device)
        return self


# Toy widths with SD-1.5's block structure, for golden vectors and CPU tests.  8 GroupNorm
# groups and 128² inputs keep it well conditioned (at 64² with 32 groups the 1×1 bottleneck
# normalises 2 values per group and a 1e-6 input change moves the maps by 1e-3).
TINY_CONFIG = dict(unet=dict(block_out_channels=(32, 64, 64, 64), cross_attention_dim=32, norm_num_groups=8),
                   vae=dict(block_out_channels=(32, 32, 64, 64), norm_num_groups=8))
TINY_IMAGE = 128


# Toy SDXL (same structure: no attention at the top level, depth-2/-N transformers, linear
# projections, text_time conditioning) for tests.
TINY_SDXL_CONFIG = dict(unet=dict(block_out_channels=(32, 64, 64), transformer_depth=(0, 1, 2), head_dim=16,
                                  cross_attention_dim=32, addition_time_embed_dim=8, pooled_dim=32, norm_num_groups=8),
                        vae=dict(block_out_channels=(32, 32, 64, 64), norm_num_groups=8))


def build_sd15(seed=0, device="cpu", weights=None, config=None, unet_cls=None):
    """Random-init SD-1.5 parts (seeded), or load a local diffusers-0.8.0 state dict.

    ``weights`` may be a directory holding ``unet.safetensors``/``vae.safetensors`` or
    ``.pt`` files (loaded with ``weights_only=True``), or a diffusers pipeline directory
    (``unet/diffusion_pytorch_model.safetensors`` …); missing files raise.  ``config`` shrinks the
    architecture (``TINY_CONFIG`` keeps SD-1.5's block structure at toy widths for
    golden vectors and CPU tests).
    """
    import os
    import torch
    g = torch.random.fork_rng(devices=[])
    with g:
        torch.manual_seed(seed)
        cfg = config or {}
        unet = (unet_cls or UNet2DConditionModel)(**cfg.get("unet", {}))
        vae = AutoencoderKL(**cfg.get("vae", {}))
    if weights:
        for name, mod in (("unet", unet), ("vae", vae)):
            cands = [os.path.join(weights, name + ext) for ext in (".safetensors", ".pt", ".bin")]
            # the diffusers pipeline layout (a Hugging Face snapshot): <name>/diffusion_pytorch_model.*
            cands += [os.path.join(weights, name, "diffusion_pytorch_model" + ext) for ext in (".safetensors", ".bin")]
            found = [p for p in cands if os.path.exists(p)]
            if not found:
                raise FileNotFoundError(f"no {name} weights in {weights} (looked for {', '.join(cands)})")
            p = found[0]
            if p.endswith(".safetensors"):
                from safetensors.torch import load_file
                sd = load_file(p)
            else:
                sd = torch.load(p, map_location="cpu", weights_only=True)
            if name == "vae":
                sd = {k: v for k, v in sd.items() if k.startswith(("encoder.", "quant_conv."))}
            mod.load_state_dict(sd, strict=True)
    sched = DDIMScheduler(beta_start=0.00085, beta_end=0.012, beta_schedule="scaled_linear",
                          clip_sample=False, set_alpha_to_one=False)
    sched.set_timesteps(50)
    for m in (unet, vae):
        m.eval()
        for p in m.parameters():
            p.requires_grad = False
    return StableDiffusionParts(unet, vae, sched).to(device)


def build_sdxl(seed=0, device="cpu", weights=None, config=None):
    """Random-init (seeded) or local-weights SDXL UNet + VAE encoder + DDIM (scaled_linear
    0.00085 → 0.012, as SD-1.5; SDXL's scheduler config uses the same betas)."""
    return build_sd15(seed=seed, device=device, weights=weights, config=config, unet_cls=SDXLUNet)
