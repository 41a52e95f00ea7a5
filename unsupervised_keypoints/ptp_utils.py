"""Alias: ``unsupervised_keypoints.ptp_utils`` is ``stablekeypoints_amd.ptp_utils`` (reference ``unsupervised_keypoints/ptp_utils.py``)."""
import sys

from stablekeypoints_amd import ptp_utils as _impl

sys.modules[__name__] = _impl
