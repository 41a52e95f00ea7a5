"""Alias: ``unsupervised_keypoints.optimize`` is ``stablekeypoints_amd.optimize`` (reference ``unsupervised_keypoints/optimize.py``)."""
import sys

from stablekeypoints_amd import optimize as _impl

sys.modules[__name__] = _impl
