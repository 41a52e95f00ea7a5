"""Alias: ``unsupervised_keypoints.eval`` is ``stablekeypoints_amd.eval`` (reference ``unsupervised_keypoints/eval.py``)."""
import sys

from stablekeypoints_amd import eval as _impl

sys.modules[__name__] = _impl
