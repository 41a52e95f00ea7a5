"""Alias for the reference's ``unsupervised_keypoints/sdxl_monkey_patch.py``.

The reference module defines ``AttentionControl``, ``AttentionStore`` and
``register_attention_control`` for SDXL-era diffusers; it never patches anything (it looks for
``AttnProcessor2_0`` among ``children()``, which processors are not).  Here SDXL capture is the
same hook as SD-1.5 (``sd/sdxl.py`` keeps the ``CrossAttention`` class name), so these names are
the ``ptp_utils`` ones and work on an SDXL UNet built by ``load_ldm(dev, "random-xl" | weights)``.
"""
from stablekeypoints_amd.ptp_utils import AttentionControl, AttentionStore, register_attention_control  # noqa: F401
