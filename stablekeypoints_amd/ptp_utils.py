"""Attention capture hook, store and token selection (mirror of reference ``ptp_utils.py``).

Same names, signatures and semantics as the reference; the capture branch, the
aggregation it feeds and the selection heuristics run as HIP kernels (libskp).

Capture algebra: the reference recomputes
``softmax(to_q(bicubic(x)) kᵀ·scale)`` at R×R (``ptp_utils.py:513-536``).
bicubic and to_q are linear and commute with ·kᵀ, so this equals
``softmax(bicubic(q kᵀ·scale))`` where ``q kᵀ·scale`` is the layer's own
normal-path logit matrix at s×s.  The patched forward therefore computes the
logits once on the matrix cores (``skp_bgemm_f32``), feeds them to the normal
softmax·V path, and hands them to the capture kernels: ≈248 GFLOP of dense work per
capture in the reference becomes ≈1.6 GFLOP of MFMA plus the upsample/softmax/aggregate
kernel ``skp_capture_maps_fwd`` (VALU-bound: 4 taps, an exp and the normalised
accumulate per (pixel, token, layer, head)), or ``skp_capture_fwd`` for
a plain ``AttentionStore``.
"""
import abc
import contextlib
import os

import numpy as np
import torch
import torch.nn as nn

from . import ops
from .sd.unet import CaptureComplete, _shared_context, attention_core, kv_projection, shared_kv


# --------------------------------------------------------------------------- A2 controller / store
class AttentionControl(abc.ABC):
    """ptp_utils.py:32-60."""

    def step_callback(self, x_t):
        return x_t

    def between_steps(self):
        return

    @property
    def num_uncond_att_layers(self):
        return 0

    @abc.abstractmethod
    def forward(self, dict, is_cross: bool, place_in_unet: str):
        raise NotImplementedError

    def __call__(self, dict, is_cross: bool, place_in_unet: str):
        dict = self.forward(dict, is_cross, place_in_unet)
        return dict["attn"]

    def reset(self):
        self.cur_step = 0
        self.cur_att_layer = 0

    def __init__(self):
        self.cur_step = 0
        self.num_att_layers = -1
        self.cur_att_layer = 0


class AttentionStore(AttentionControl):
    """ptp_utils.py:63-83: ``step_store["attn"]`` lists captured (B·H, R², N) maps in order.

    ``early_exit`` (default False = reference behaviour): when True, the patched
    attention raises ``CaptureComplete`` once the 4th map is stored, so the UNet
    forward stops there; the reference discards that forward's output anyway
    (``ptp_utils.py:246-252``) and nothing later feeds the loss.

    ``stores_logits`` (class default False): when set, the hook hands the store each captured
    layer's low-resolution logits (B·H, s², N) with their grid side instead of the (B·H, R², N)
    attention; ``maps_per_image`` then builds maps with the fused capture.  ``LogitStore`` sets
    it for good; ``logit_capture`` sets it on an ``AttentionStore`` for one capture pass whose
    maps the caller collects at once (``run_and_find_attn``).
    """

    max_captures = 4
    stores_logits = False

    @staticmethod
    def get_empty_store():
        return {"attn": []}

    def forward(self, dict, is_cross: bool, place_in_unet: str):
        self.step_store["attn"].append(dict["attn"])
        if "size" in dict:
            self.step_store.setdefault("size", []).append(dict["size"])
            self.heads = dict.get("heads", getattr(self, "heads", 8))
        return dict

    def reset(self):
        super().reset()
        self.step_store = self.get_empty_store()

    def __init__(self, early_exit=False):
        super().__init__()
        self.step_store = self.get_empty_store()
        self.early_exit = early_exit

    def maps_per_image(self, B, R, layers=(0, 1, 2, 3), captured=False):
        """(B, N, R, R) maps of the stored logits (CaptureMaps, dense backward), or with
        ``captured`` an ``ops.CapturedMaps`` whose ``select`` gathers rows with the sparse
        backward.  Needs a store that holds logits (``stores_logits``)."""
        zs = [z for li, z in enumerate(self.step_store["attn"]) if li in layers]
        ss = [sz for li, sz in enumerate(self.step_store.get("size", [])) if li in layers]
        if not zs:
            raise RuntimeError("maps_per_image: no captured layers (is the hook registered?)")
        if len(ss) != len(zs):
            raise RuntimeError("maps_per_image: the store holds attention, not logits (stores_logits unset)")
        if captured:
            return ops.CapturedMaps(zs, ss, B, R)
        return ops.capture_maps(zs, ss, B, R)


class LogitStore(AttentionStore):
    """Fast-path store: keeps each captured layer's low-resolution logits (B·H, s², N)
    instead of the (B·H, R², N) attention; maps are produced by the fused
    ``ops.capture_maps`` (per image) when collected, and the backward never
    materialises a (B·H, R², N) gradient.  ``step_store["attn"]`` holds the logits and
    ``step_store["size"]`` the grid side s of each."""

    stores_logits = True

    @staticmethod
    def get_empty_store():
        return {"attn": [], "size": []}


# A/B: 0 = run_and_find_attn fills an AttentionStore with the materialised (B·H, R², N)
# attention of every captured layer, as in r02
EVAL_LOGITS = True   # tests switch it: False = the AttentionStore capture path


@contextlib.contextmanager
def logit_capture(controllers):
    """Capture LOGITS into the given ``AttentionStore``s for one pass whose maps the caller
    collects before the block ends (``run_and_find_attn`` / ``run_and_find_attn_per_image``).

    The reference stores the (B·H, R², N) attention of every captured layer (1.05 GB per
    layer at N=500, R=128, B·H=8; ptp_utils.py:508-538) and ``collect_maps`` immediately
    reduces it to the (N', R', R') map (optimize.py:27-79); here the same maps come from the
    fused ``skp_capture_maps_fwd`` over the stored (B·H, s², N) logits, and nothing of size
    (B·H, R², N) is written.  Stores that already hold logits, stores of another class and
    non-store controllers are left alone.  On exit every switched store is reset (the
    reference's callers reset after collecting) and switched back."""
    switched = []
    if EVAL_LOGITS:
        for ctl in controllers.values():
            if type(ctl) is AttentionStore and not ctl.stores_logits and not ctl.step_store["attn"]:
                ctl.stores_logits = True
                switched.append(ctl)
    try:
        yield
    finally:
        for ctl in switched:
            del ctl.stores_logits
            ctl.reset()


# --------------------------------------------------------------------------- A1 capture hook
def register_attention_control(model, controller, feature_upsample_res=256):
    """ptp_utils.py:472-573: patch every ``CrossAttention`` under children named "*up*"."""

    def ca_forward(self, place_in_unet):
        to_out = self.to_out
        if type(to_out) is torch.nn.modules.container.ModuleList:
            to_out = self.to_out[0]

        def forward(x, context=None, mask=None):
            batch_size, sequence_length, dim = x.shape
            h = self.heads
            is_cross = context is not None
            capture = (is_cross and sequence_length <= 32 ** 2
                       and len(controller.step_store["attn"]) < AttentionStore.max_captures)
            if not capture:
                # ptp_utils.py:481-506: un-captured layers are the normal attention (the class's own
                # forward: projections read in place, fused attention)
                return type(self).forward(self, x, context, mask)
            q = self.to_q(x)
            one = _shared_context(context) if (is_cross and mask is None and x.is_cuda) else None
            # the shared embedding's k / v projected once (its (1, N, H·d) projections decide eligibility)
            k1, v1 = shared_kv(self, one) if (capture and one is not None) else (None, None)
            if k1 is not None and ops.heads_eligible(q, k1, h):
                # the capture on the layer's own (B, S, H·d) projection and the ONE projection of the
                # token embedding the batch shares: no head permutes, no batch-expanded keys / values
                s = int(sequence_length ** 0.5)
                if s * s != sequence_length:
                    raise ValueError(f"capture needs a square token grid, got {sequence_length}")
                sim = ops.capture_logits_heads(q, k1, h, self.scale)      # (B·H, s², N), MFMA
                if getattr(controller, "stores_logits", False):
                    controller({"attn": sim, "size": s, "heads": h}, is_cross, place_in_unet)
                else:
                    attn = ops.capture_attn(sim, s, feature_upsample_res)  # (B·H, R², N), HIP
                    controller({"attn": attn}, is_cross, place_in_unet)
                if getattr(controller, "early_exit", False) and \
                        len(controller.step_store["attn"]) >= AttentionStore.max_captures:
                    raise CaptureComplete()   # the UNet output is discarded: skip this layer's output too
                return to_out(ops.attn_pv_heads(sim.softmax(dim=-1), v1, h))
            context = context if is_cross else x
            if k1 is not None:
                k, v = k1.expand(batch_size, -1, -1), v1.expand(batch_size, -1, -1)
            else:
                k, v = kv_projection(self, context)
            q = self.reshape_heads_to_batch_dim(q)
            k = self.reshape_heads_to_batch_dim(k)
            v = self.reshape_heads_to_batch_dim(v)
            if capture:
                s = int(sequence_length ** 0.5)
                if s * s != sequence_length:
                    raise ValueError(f"capture needs a square token grid, got {sequence_length}")
                sim = ops.capture_logits(q, k, self.scale)          # (B·H, s², N), MFMA
                sim_n = sim
                if mask is not None:   # the mask applies to the normal path only (ptp_utils.py:496-500)
                    m = mask.reshape(batch_size, -1)[:, None, :].repeat(h, 1, 1)
                    sim_n = sim.masked_fill(~m, -torch.finfo(sim.dtype).max)
                out = torch.bmm(sim_n.softmax(dim=-1), v)
                if getattr(controller, "stores_logits", False):
                    controller({"attn": sim, "size": s, "heads": h}, is_cross, place_in_unet)
                else:
                    attn = ops.capture_attn(sim, s, feature_upsample_res)  # (B·H, R², N), HIP
                    controller({"attn": attn}, is_cross, place_in_unet)
            else:
                out = attention_core(q, k, v, self.scale, mask, h)
            out = to_out(self.reshape_batch_dim_to_heads(out))
            if capture and getattr(controller, "early_exit", False) and \
                    len(controller.step_store["attn"]) >= AttentionStore.max_captures:
                raise CaptureComplete()
            return out

        return forward

    class DummyController:
        def __call__(self, *args):
            return args[0]

        def __init__(self):
            self.num_att_layers = 0
            self.step_store = {"attn": []}

    if controller is None:
        controller = DummyController()

    def register_recr(net_, count, place_in_unet):
        if net_.__class__.__name__ == "CrossAttention":
            net_.forward = ca_forward(net_, place_in_unet)
            return count + 1
        elif hasattr(net_, "children"):
            for net__ in net_.children():
                count = register_recr(net__, count, place_in_unet)
        return count

    if not isinstance(controller, DummyController):
        controller.feature_upsample_res = feature_upsample_res   # R of the logit-store maps
    cross_att_count = 0
    for name, net in model.named_children():
        if "up" in name:
            cross_att_count += register_recr(net, 0, "up")
    controller.num_att_layers = cross_att_count
    assert cross_att_count != 0, "No cross attention layers found in the model. Please check to make sure " \
                                 "you're using diffusers==0.8.0."


# --------------------------------------------------------------------------- A8-A10 selection
def find_top_k_gaussian(attention_maps, top_k, sigma=3, epsilon=1e-5, num_subjects=1):
    """ptp_utils.py:86-112 (skp_topk_gaussian)."""
    return ops.find_top_k_gaussian(attention_maps, top_k, sigma=sigma, epsilon=epsilon, num_subjects=num_subjects)


def furthest_point_sampling(attention_maps, top_k, top_initial_candidates):
    """ptp_utils.py:115-159 (skp_fps).  Returns the selected token ids (int64, device)."""
    sel, n = ops.furthest_point_sampling(attention_maps, top_k, top_initial_candidates)
    if top_k > len(top_initial_candidates):   # the reference returns fewer when candidates run out
        return sel[: int(n.item())]
    return sel


def entropy_sort(attention_maps, top_k, min_dist=0.05):
    """ptp_utils.py:165-187 (skp_entropy_sort)."""
    return ops.entropy_sort(attention_maps, top_k)


def random_range(size, min_val, max_val, dtype=torch.float32):
    return torch.rand(size, dtype=dtype) * (max_val - min_val) + min_val


# --------------------------------------------------------------------------- A14 capture driver
def image2latent(model, image, device):
    """ptp_utils.py:289-304: (2x−1) → VAE encoder mean · 0.18215 (kept on the device)."""
    with torch.no_grad():
        if isinstance(image, np.ndarray):
            image = torch.from_numpy(image).float().permute(0, 3, 1, 2)
        if image.dim() == 4 and image.shape[1] == 4:   # already a latent
            return image.to(device)
        image = image.to(device, torch.float32) * 2 - 1
        vae = model.vae.module if isinstance(model.vae, nn.DataParallel) else model.vae
        return vae.encode(image)["latent_dist"].mean * 0.18215


def find_pred_noise(ldm, image, context, noise_level=-1, device="cuda"):
    """ptp_utils.py:205-231.  The UNet output is None when the store stops the forward early."""
    with torch.no_grad():
        latent = image2latent(ldm, image, device)
    noise = torch.randn_like(latent)
    t = ldm.scheduler.timesteps[noise_level]
    if t.device != latent.device:
        # the timestep made on the device (a fill), not uploaded: a pageable host-to-device copy
        # waits for the whole queued stream and stalls the host at every capture
        t = torch.full((), int(t), dtype=t.dtype, device=latent.device)
    noisy_image = ldm.scheduler.add_noise(latent, noise, t)
    try:
        # the reference repeats the context per image; a stride-0 expansion is the same tensor
        # to every consumer, and lets the cross-attention project it once (unet.kv_projection)
        B = noisy_image.shape[0]
        ctx = context.expand(B, -1, -1) if context.shape[0] == 1 else context.repeat(B, 1, 1)
        pred_noise = ldm.unet(noisy_image, t.repeat(B), ctx)["sample"]
    except CaptureComplete:
        pred_noise = None
    return noise, pred_noise


def run_and_find_attn(ldm, image, context, noise_level=-1, device="cuda",
                      from_where=("down_cross", "mid_cross", "up_cross"), layers=(0, 1, 2, 3, 4, 5),
                      upsample_res=32, indices=None, controllers=None):
    """ptp_utils.py:234-272: one UNet pass, then collect_maps + reset per controller."""
    from .optimize import collect_maps
    attention_maps = []
    with logit_capture(controllers):   # same maps, no (B·H, R², N) attention written
        find_pred_noise(ldm, image, context, noise_level=noise_level, device=device)
        for controller in controllers:
            attention_maps.append(collect_maps(controllers[controller], from_where=from_where,
                                               upsample_res=upsample_res, layers=layers, indices=indices))
            controllers[controller].reset()
    return attention_maps


def run_and_find_attn_per_image(ldm, images, context, noise_level=-1, device="cuda", layers=(0, 1, 2, 3),
                                upsample_res=-1, indices=None, controllers=None, stacked=False, captured=False):
    """Batched capture: ONE VAE + UNet pass over B images, maps aggregated PER IMAGE.

    Equivalent to B calls of ``run_and_find_attn`` with one image each (every UNet/VAE op is
    per-sample; each image gets its own noise draw), but at batch B on the GPU.  The
    reference's ``collect_maps`` averages over B·heads (optimize.py:75), which would mix
    images at B > 1, so each image's (H, R², N) slice of the stored layers is aggregated
    separately.  Returns a list (per controller) of lists (per image) of (N', R', R') maps;
    with ``stacked`` (logit store, no ``indices``/``upsample_res``) one (B, N, R, R) tensor per
    controller instead, so callers can gather rows of several images in one autograd op.
    """
    with logit_capture(controllers):   # same maps, no (B·H, R², N) attention written
        return _collect_per_image(ldm, images, context, noise_level, device, layers, upsample_res, indices,
                                  controllers, stacked, captured)


def _collect_per_image(ldm, images, context, noise_level, device, layers, upsample_res, indices, controllers,
                       stacked, captured):
    find_pred_noise(ldm, images, context, noise_level=noise_level, device=device)
    B = images.shape[0]
    out = []
    for key in controllers:
        ctl = controllers[key]
        if getattr(ctl, "stores_logits", False):
            if captured:
                out.append(ctl.maps_per_image(B, ldm.feature_upsample_res, layers, captured=True))
                ctl.reset()
                continue
            maps = ctl.maps_per_image(B, ldm.feature_upsample_res, layers)
            if stacked and indices is None:
                if upsample_res not in (-1, maps.shape[-1]):   # every image's maps in one resize launch
                    Bm, Nm, R = maps.shape[:3]
                    maps = ops.resize_bilinear(maps.view(Bm * Nm, R, R), upsample_res).view(
                        Bm, Nm, upsample_res, upsample_res)
                out.append(maps)
                ctl.reset()
                continue
            res = []
            for b in range(B):
                m = maps[b]
                if indices is not None:
                    m = m[torch.as_tensor(indices, device=m.device)]
                if upsample_res != -1 and upsample_res != m.shape[-1]:
                    m = ops.resize_bilinear(m, upsample_res)
                res.append(m)
            out.append(res)
            ctl.reset()
            continue
        stored = [a for li, a in enumerate(ctl.step_store["attn"]) if li in layers]
        if not stored:
            raise RuntimeError("no captured attention maps (is the hook registered?)")
        H = stored[0].shape[0] // B
        idx = None if indices is None else torch.as_tensor(indices, dtype=torch.int64)
        out.append([ops.aggregate([a[b * H:(b + 1) * H] for a in stored], indices=idx, upsample_res=upsample_res)
                    for b in range(B)])
        ctl.reset()
    return out


def init_random_noise(device, num_words=77, dim=768):
    """ptp_utils.py:649-650 (CPU RNG, then moved), ``dim`` generalises the hard-coded 768."""
    return torch.randn(1, num_words, dim).to(device)
