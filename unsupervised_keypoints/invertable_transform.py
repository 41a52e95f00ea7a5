"""Alias: ``unsupervised_keypoints.invertable_transform`` is ``stablekeypoints_amd.invertable_transform`` (reference ``unsupervised_keypoints/invertable_transform.py``)."""
import sys

from stablekeypoints_amd import invertable_transform as _impl

sys.modules[__name__] = _impl
