"""Alias: ``unsupervised_keypoints.main`` is ``stablekeypoints_amd.main`` (reference
``unsupervised_keypoints/main.py``); ``python -m unsupervised_keypoints.main <flags>`` runs its CLI."""
import sys

from stablekeypoints_amd import main as _impl

if __name__ == "__main__":
    _impl.main()
else:
    sys.modules[__name__] = _impl
