"""Model loading and Gaussian targets (mirror of reference ``optimize_token.py``).

``load_ldm`` keeps the reference signature and return value
``(ldm, controllers, num_gpus)`` (``optimize_token.py:24-79``), MI355X-style:
- no ``nn.DataParallel``: one process per GPU; ``controllers`` holds the single
  ``AttentionStore`` of this process's device and ``num_gpus`` is the world size;
- no network: ``type`` names a local directory of diffusers-0.8.0 UNet/VAE
  weights (``unet.safetensors``/``vae.safetensors``/``.pt``); any other value
  (e.g. the reference's hub name) builds the SD-1.5 architecture with seeded
  random weights, which is what the benchmarks use.
"""
import os

import torch

from . import ops, ptp_utils
from .sd import build_sd15, build_sdxl


def _world():
    import torch.distributed as dist
    if dist.is_available() and dist.is_initialized():
        return dist.get_world_size()
    return 1


def load_ldm(device, type="CompVis/stable-diffusion-v1-4", feature_upsample_res=256, seed=0, config=None,
             early_exit=True):
    """optimize_token.py:24-79.

    ``early_exit`` lets the patched attention stop the UNet forward after the 4th
    capture (the reference discards that output; DESIGN.md §UNet early exit).
    """
    weights = type if (isinstance(type, str) and os.path.isdir(type)) else None
    xl = isinstance(type, str) and ("xl" in type.lower())   # SDXL
    if type == "tiny" and config is None:   # toy-width SD-1.5 (tests, CLI smoke runs)
        from .sd import TINY_CONFIG
        config = TINY_CONFIG
    if type == "tiny-xl" and config is None:
        from .sd import TINY_SDXL_CONFIG
        config = TINY_SDXL_CONFIG
    if weights is None and str(device) != "cpu":
        pass  # hub names cannot be fetched offline: random-init SD-1.5 (seeded) instead
    ldm = (build_sdxl if xl else build_sd15)(seed=seed, device=device, weights=weights, config=config)
    dev = torch.device(device)
    if dev.type == "cuda":
        from .tuning import use_tuned_gemms
        use_tuned_gemms()   # measured hipBLASLt / rocBLAS choices for the UNet/VAE GEMM shapes
    if dev.type == "cuda" and dev.index is None:
        dev = torch.device("cuda", torch.cuda.current_device())
    controllers = {dev: ptp_utils.AttentionStore(early_exit=early_exit)}
    ptp_utils.register_attention_control(ldm.unet, controllers[dev], feature_upsample_res=feature_upsample_res)

    def hook_fn(module, inp):   # optimize_token.py:59-68: route each forward to its device's store
        d = inp[0].device
        if d not in controllers:
            raise RuntimeError(f"UNet input on {d}, but this process's controller is on {list(controllers)}")
    ldm.unet.register_forward_pre_hook(hook_fn)
    ldm.feature_upsample_res = feature_upsample_res
    return ldm, controllers, _world()


def gaussian_circle(pos, size=64, sigma=16, device="cuda"):
    """optimize_token.py:204-224: pos (T, 2) in [0, 1] -> (T, size, size) (skp_gaussian_target)."""
    return ops.gaussian_circles(pos.to(device).unsqueeze(0), size, sigma)


def gaussian_circles(pos, size=64, sigma=16, device="cuda"):
    """optimize_token.py:226-242: pos (num, T, 2) -> mean over the num circles (skp_gaussian_target)."""
    return ops.gaussian_circles(pos.to(device), size, sigma)
