"""Alias for the reference's ``unsupervised_keypoints/sdxl_monkey_patch.py``: its
SDXL-era store API (``AttentionControl`` / ``AttentionStore`` with per-place keys, the 32² filter,
the conditional half, ``between_steps`` / ``get_average_attention``) and a
``register_attention_control`` that feeds it from this package's SDXL UNet — see
``stablekeypoints_amd.sdxl_monkey_patch``."""
from stablekeypoints_amd.sdxl_monkey_patch import AttentionControl, AttentionStore, register_attention_control  # noqa: F401
