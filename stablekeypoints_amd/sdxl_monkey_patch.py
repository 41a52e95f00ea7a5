"""The SDXL-era attention store API of the reference (``unsupervised_keypoints/sdxl_monkey_patch.py``).

The reference module is a prompt-to-prompt style controller for diffusers' ``AttnProcessor2_0``
attention:

* ``AttentionControl`` (``sdxl_monkey_patch.py:8-44``): called with the attention PROBABILITIES of
  one layer, ``(batch·heads, pixels, keys)``; only the conditional half ``attn[h // 2:]`` goes
  through ``forward`` and is written back in place; a layer counter that, every
  ``num_att_layers + num_uncond_att_layers`` calls, ends a diffusion step (``cur_step``) and runs
  ``between_steps``;
* ``AttentionStore`` (``:48-86``): per-place lists (``down/mid/up`` × ``cross/self``) of the
  layers with at most 32² pixels, summed over steps in ``between_steps`` (in place, into the
  tensors of the first step), ``get_average_attention`` = that sum / ``cur_step``;
* ``register_attention_control`` (``:89-214``): inert in the reference — it looks for
  ``AttnProcessor2_0`` among ``children()`` (processors are not modules), prints "Not found",
  patches nothing and never sets ``num_att_layers``.

The two classes are restated here with the reference's members and arithmetic (pinned
bit-for-bit by ``tests/golden/sdxl_store.npz``, recorded from the reference's own class).
``register_attention_control`` here does what the reference's intends on this package's SDXL
UNet (``sd/sdxl.py``, whose attention modules keep diffusers-0.8.0's ``CrossAttention`` layout):
every attention module under the ``down`` / ``mid`` / ``up`` children computes its probabilities
``softmax(q·kᵀ·scale)``, hands them to the controller with ``(is_cross, place)`` and uses what
it returns, and ``controller.num_att_layers`` is set to the number of patched modules.  It is an
API-compatibility path (every layer's full probability tensor is materialised, as the reference's
processor would): the keypoint training path uses ``ptp_utils`` (``LogitStore`` and the fused
capture kernels) on the same UNet.
"""
import abc

import torch


class AttentionControl(abc.ABC):
    """sdxl_monkey_patch.py:8-44."""

    def __init__(self):
        self.cur_step = 0
        self.num_att_layers = -1
        self.cur_att_layer = 0

    def step_callback(self, x_t):
        return x_t

    def between_steps(self):
        return

    @property
    def num_uncond_att_layers(self):
        return 0

    @abc.abstractmethod
    def forward(self, attn, is_cross: bool, place_in_unet: str):
        raise NotImplementedError

    def __call__(self, attn, is_cross: bool, place_in_unet: str):
        # the unconditional layers are only counted; the conditional half of the batch·heads axis
        # goes through forward and is written back into attn
        if self.cur_att_layer >= self.num_uncond_att_layers:
            half = attn.shape[0] // 2
            attn[half:] = self.forward(attn[half:], is_cross, place_in_unet)
        self.cur_att_layer += 1
        if self.cur_att_layer == self.num_att_layers + self.num_uncond_att_layers:
            self.cur_att_layer = 0
            self.cur_step += 1
            self.between_steps()
        return attn

    def reset(self):
        self.cur_step = 0
        self.cur_att_layer = 0


class AttentionStore(AttentionControl):
    """sdxl_monkey_patch.py:48-86."""

    PLACES = ("down", "mid", "up")
    MAX_PIXELS = 32 ** 2   # larger layers are not kept (the reference's memory guard)

    def __init__(self):
        super().__init__()
        self.step_store = self.get_empty_store()
        self.attention_store = {}

    @staticmethod
    def get_empty_store():
        return {f"{p}_{kind}": [] for kind in ("cross", "self") for p in AttentionStore.PLACES}

    def forward(self, attn, is_cross: bool, place_in_unet: str):
        if attn.shape[1] <= self.MAX_PIXELS:
            self.step_store[f"{place_in_unet}_{'cross' if is_cross else 'self'}"].append(attn)
        return attn

    def between_steps(self):
        if not self.attention_store:
            # the first step's lists become the running sums (later steps add into those tensors)
            self.attention_store = self.step_store
        else:
            for key, maps in self.attention_store.items():
                for i in range(len(maps)):   # the running sums' length rules (a short step raises)
                    maps[i] += self.step_store[key][i]
        self.step_store = self.get_empty_store()

    def get_average_attention(self):
        return {key: [m / self.cur_step for m in maps] for key, maps in self.attention_store.items()}

    def reset(self):
        super().reset()
        self.step_store = self.get_empty_store()
        self.attention_store = {}


def _attention_module_forward(module, controller, place_in_unet):
    """The patched forward of one CrossAttention module: the layer's probabilities through the
    controller (sdxl_monkey_patch.py:25-37's protocol), then the value aggregation with what it
    returned.  Self-attention when ``context`` is None."""
    to_out = module.to_out

    def forward(x, context=None, mask=None):
        is_cross = context is not None
        ctx = x if context is None else context
        q = module.reshape_heads_to_batch_dim(module.to_q(x))
        k = module.reshape_heads_to_batch_dim(module.to_k(ctx))
        v = module.reshape_heads_to_batch_dim(module.to_v(ctx))
        scores = torch.baddbmm(torch.empty(q.shape[0], q.shape[1], k.shape[1], dtype=q.dtype, device=q.device),
                               q, k.transpose(1, 2), beta=0, alpha=module.scale)
        if mask is not None:
            scores = scores.masked_fill(~mask.bool(), -torch.finfo(scores.dtype).max)
        attn = controller(scores.softmax(dim=-1), is_cross, place_in_unet)
        out = module.reshape_batch_dim_to_heads(torch.bmm(attn, v))
        return to_out[1](to_out[0](out))

    return forward


def register_attention_control(model, controller):
    """Patch every attention module under the UNet's ``down*`` / ``mid*`` / ``up*`` children
    (sdxl_monkey_patch.py:164-214's walk, with this package's CrossAttention class in place of
    ``AttnProcessor2_0``) so that its probabilities go through ``controller``; sets
    ``controller.num_att_layers`` and returns the number of patched modules.  ``model`` is the
    ``load_ldm`` pipeline (``model.unet``) or a UNet."""
    unet = getattr(model, "unet", model)

    def walk(net, place):
        if net.__class__.__name__ == "CrossAttention":
            net.forward = _attention_module_forward(net, controller, place)
            return 1
        return sum(walk(child, place) for child in net.children())

    count = 0
    for name, net in unet.named_children():
        for place in ("down", "up", "mid"):
            if place in name:
                count += walk(net, place)
                break
    controller.num_att_layers = count
    return count
