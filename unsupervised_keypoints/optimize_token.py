"""Alias: ``unsupervised_keypoints.optimize_token`` is ``stablekeypoints_amd.optimize_token`` (reference ``unsupervised_keypoints/optimize_token.py``)."""
import sys

from stablekeypoints_amd import optimize_token as _impl

sys.modules[__name__] = _impl
