"""The reference's import path, ``unsupervised_keypoints.*`` (damaggu/StableKeypoints), resolved
to this package's modules so reference callers run unchanged:

    from unsupervised_keypoints.optimize_token import load_ldm        # reference main.py:7
    from unsupervised_keypoints.optimize import optimize_embedding    # reference main.py:8
    python -m unsupervised_keypoints.main --dataset_loc ... --model_type <weights dir>

Each submodule IS the ``stablekeypoints_amd`` module of the same name (``sys.modules`` alias: the
same objects, so monkey-patching one patches the other).  ``sdxl_monkey_patch`` is the restated
SDXL store API (``AttentionControl`` / ``AttentionStore``, pinned by a fixture recorded from the
reference's classes) with ``register_attention_control`` on this package's SDXL UNet (the
reference's own patch patches nothing).  Not built: ``visualize``
(matplotlib figures), ``generate_image`` (text-to-image), ``cub`` (h5py): importing them raises
ImportError.
"""
