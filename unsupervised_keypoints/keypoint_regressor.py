"""Alias: ``unsupervised_keypoints.keypoint_regressor`` is ``stablekeypoints_amd.keypoint_regressor`` (reference ``unsupervised_keypoints/keypoint_regressor.py``)."""
import sys

from stablekeypoints_amd import keypoint_regressor as _impl

sys.modules[__name__] = _impl
