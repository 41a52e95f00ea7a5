"""stablekeypoints_amd — MI355X-native hot path of StableKeypoints.

Reference-mirroring modules (same names/signatures as damaggu/StableKeypoints'
``unsupervised_keypoints``): ``ptp_utils``, ``optimize``, ``optimize_token``,
``eval``, ``invertable_transform``, ``main``.  The hot path runs as HIP kernels in
``libskp.so`` (C ABI: ``include/skp.h``; binding: ``_lib``; autograd ops: ``ops``);
the frozen SD-1.5 UNet/VAE (``sd``) stays in PyTorch-ROCm.
"""
__version__ = "0.1.0"
