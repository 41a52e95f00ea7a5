"""Model loading and Gaussian targets (mirror of reference ``optimize_token.py``).

``load_ldm`` keeps the reference signature and return value
``(ldm, controllers, num_gpus)`` (``optimize_token.py:24-79``), MI355X-style:
- no ``nn.DataParallel``: one process per GPU; ``controllers`` holds the single
  ``AttentionStore`` of this process's device and ``num_gpus`` is the world size;
- no network.  ``type`` is resolved by ``resolve_model``: a local weight directory, a hub
  name already present in the local Hugging Face cache, or an explicit random-init name
  (``"random"``, ``"random-xl"``, ``"tiny"``, ``"tiny-xl"``).  Anything else raises
  ``ModelNotAvailableError``: the reference's default names never silently become random
  weights.
"""
import os

import torch

from . import ops, ptp_utils
from .sd import build_sd15, build_sdxl

# explicit random-init model names -> (SDXL?, tiny config?)
RANDOM_MODELS = {"random": (False, False), "random-xl": (True, False), "tiny": (False, True),
                 "tiny-xl": (True, True)}


# Hugging Face cache to resolve hub names in (None: huggingface_hub's default, HF_HUB_CACHE / HF_HOME)
HF_CACHE_DIR = None


class ModelNotAvailableError(FileNotFoundError):
    """``load_ldm`` was given a model it cannot load offline (not a local directory, not in the
    local Hugging Face cache, not an explicit random-init name)."""


def _world():
    import torch.distributed as dist
    if dist.is_available() and dist.is_initialized():
        return dist.get_world_size()
    return 1


def _hub_snapshot(name):
    """The local snapshot directory of hub repo ``name`` if the Hugging Face cache holds it
    (``local_files_only``: never touches the network), else None."""
    if "/" not in name or name.count("/") != 1:
        return None
    try:
        from huggingface_hub import snapshot_download
    except ImportError:
        return None
    try:
        return snapshot_download(name, local_files_only=True, cache_dir=HF_CACHE_DIR)
    except Exception:   # LocalEntryNotFoundError, a malformed id, a broken cache: not available
        return None


# diffusers config.json keys that map one-to-one onto this package's SD-1.5 constructors
_UNET_KEYS = ("in_channels", "out_channels", "block_out_channels", "cross_attention_dim", "attention_head_dim",
              "norm_num_groups")
_VAE_KEYS = ("block_out_channels", "latent_channels", "norm_num_groups")


def _snapshot_model(path, xl):
    """(path, is_sdxl, architecture config) of a weight directory.  A diffusers pipeline layout
    carries ``unet/config.json`` and ``vae/config.json``: the UNet's cross-attention width decides
    SDXL (2048) vs the SD-1.x family, whose block widths, head count, groups and channels are
    taken from the files (SDXL keeps the base-1.0 architecture of ``sd.SDXL_CONFIG``)."""
    import json
    cfgs = {}
    for part in ("unet", "vae"):
        p = os.path.join(path, part, "config.json")
        if os.path.exists(p):
            with open(p) as f:
                cfgs[part] = json.load(f)
    if "unet" in cfgs:
        xl = cfgs["unet"].get("cross_attention_dim") == 2048
    if xl or not cfgs:
        return path, xl, None
    arch = {}
    for part, keys in (("unet", _UNET_KEYS), ("vae", _VAE_KEYS)):
        if part in cfgs:
            arch[part] = {k: (tuple(v) if isinstance(v, list) else v) for k, v in cfgs[part].items() if k in keys}
    return path, xl, arch


def resolve_model(type):
    """(weights directory or None, is_sdxl, architecture config or None) for ``load_ldm``'s ``type``.

    - a local directory: its weights (``unet.safetensors`` / ``.pt`` / ``.bin`` or the diffusers
      pipeline layout ``unet/diffusion_pytorch_model.*``; see ``sd.build_sd15``);
    - a hub name (``"runwayml/stable-diffusion-v1-5"``): its snapshot in the local Hugging Face
      cache, if present;
    - ``"random"`` / ``"random-xl"``: SD-1.5 / SDXL with seeded random weights (benchmarks);
      ``"tiny"`` / ``"tiny-xl"``: the toy-width models of the tests;
    - otherwise ``ModelNotAvailableError``.
    SDXL is chosen by a name containing "xl" (``stabilityai/stable-diffusion-xl-base-1.0``).
    """
    if not isinstance(type, (str, os.PathLike)):
        raise TypeError(f"load_ldm: model type must be a string or path, got {type!r}")
    type = os.fspath(type)
    if type in RANDOM_MODELS:
        xl, tiny = RANDOM_MODELS[type]
        cfg = None
        if tiny:
            from .sd import TINY_CONFIG, TINY_SDXL_CONFIG
            cfg = TINY_SDXL_CONFIG if xl else TINY_CONFIG
        return None, xl, cfg
    xl = "xl" in os.path.basename(type.rstrip("/")).lower()
    path = os.path.expanduser(type)
    snap = path if os.path.isdir(path) else _hub_snapshot(type)
    if snap is not None:
        return _snapshot_model(snap, xl)
    raise ModelNotAvailableError(
        f"load_ldm: cannot load model {type!r}: it is not a local directory and not in the local Hugging Face "
        "cache, and this build never downloads. Pass a directory of diffusers-0.8.0 UNet/VAE weights, or "
        "type='random' (SD-1.5) / 'random-xl' (SDXL) for seeded random weights.")


def load_ldm(device, type="CompVis/stable-diffusion-v1-4", feature_upsample_res=256, seed=0, config=None,
             early_exit=True):
    """optimize_token.py:24-79.

    ``type``: see ``resolve_model`` (raises ``ModelNotAvailableError`` for a model it cannot load;
    the reference would download it).  ``config`` overrides the architecture of a random-init
    model (tests).  ``early_exit`` lets the patched attention stop the UNet forward after the 4th
    capture (the reference discards that output; DESIGN.md §UNet early exit).
    """
    weights, xl, cfg = resolve_model(type)
    if config is not None:
        if weights is not None:
            raise ValueError("load_ldm: `config` only applies to random-init models, not to loaded weights")
        cfg = config
    ldm = (build_sdxl if xl else build_sd15)(seed=seed, device=device, weights=weights, config=cfg)
    ldm.model_type = type
    dev = torch.device(device)
    if dev.type == "cuda" and dev.index is None:
        dev = torch.device("cuda", torch.cuda.current_device())
    if dev.type == "cuda":
        from .tuning import use_tuned_gemms
        use_tuned_gemms(dev)   # measured hipBLASLt / rocBLAS choices for the UNet/VAE GEMM shapes
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
