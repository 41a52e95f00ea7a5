"""Keypoint extraction: argmax / soft-argmax and test-time augmentation (mirror of reference ``eval.py``).

``find_max_pixel``, ``find_k_max_pixels``, ``mask_radius`` and
``pixel_from_weighted_avg`` (``eval.py:39-155``) run as HIP kernels with the
reference's semantics (first-occurrence argmax, NaN is max, in-place mutation in
``pixel_from_weighted_avg``).  Dataset metrics (``evaluate``, ``eval.py:374-539``)
are outside the hot path and not part of this package.
"""
import torch

from . import ops, ptp_utils
from .invertable_transform import RandomAffineWithInverse


def find_max_pixel(map):
    """eval.py:39-60: (T, h, w) -> (T, 2) float (row + 0.5, col + 0.5)."""
    return ops.find_max_pixel(map)


def find_k_max_pixels(map, num=3):
    """eval.py:62-81: (num, T, 2)."""
    return ops.find_k_max_pixels(map, num=num)


def mask_radius(map, max_coords, radius):
    """eval.py:83-111."""
    return ops.mask_radius(map, max_coords, radius)


def pixel_from_weighted_avg(heatmaps, distance=5):
    """eval.py:113-155 (zeros pixels beyond ``distance`` IN PLACE, like the reference)."""
    return ops.pixel_from_weighted_avg(heatmaps, distance=distance)


@torch.no_grad()
def run_image_with_context_augmented(ldm, image, context, indices, device="cuda",
                                     from_where=("down_cross", "mid_cross", "up_cross"), layers=(0, 1, 2, 3, 4, 5),
                                     augmentation_iterations=20, noise_level=-1, augment_degrees=30,
                                     augment_scale=(0.9, 1.1), augment_translate=(0.1, 0.1), visualize=False,
                                     controllers=None, num_gpus=1, save_folder="outputs", upscale_size=512):
    """eval.py:197-355 (hot part 221-266, 327-330): TTA-averaged maps of the chosen tokens.

    ``image`` is (3, H, W) in [0, 1].  Each iteration warps ``num_gpus`` copies
    (on this process: one copy per iteration), captures, gathers ``indices`` and
    bilinearly upsamples to ``upscale_size`` (collect_maps), inverse-warps maps and
    ones and accumulates; returns sum / count with NaN -> 0.
    """
    if visualize:
        raise NotImplementedError("visualisation is outside the hot path")
    img = image if torch.is_tensor(image) else torch.as_tensor(image)
    if img.dim() == 3 and img.shape[-1] == 3 and img.shape[0] != 3:
        img = img.permute(2, 0, 1)
    img = img.to(device, torch.float32)
    n = len(indices)
    num_samples = torch.zeros(n, upscale_size, upscale_size, device=device)
    sum_samples = torch.zeros(n, upscale_size, upscale_size, device=device)
    T = RandomAffineWithInverse(degrees=augment_degrees, scale=augment_scale, translate=augment_translate)
    for _ in range(augmentation_iterations // num_gpus):
        aug = T(img[None])
        maps = ptp_utils.run_and_find_attn(ldm, aug, context, layers=layers, noise_level=noise_level,
                                           from_where=from_where, upsample_res=upscale_size, device=device,
                                           controllers=controllers, indices=indices)
        maps = torch.stack(maps)          # (1, n, S, S) on this rank
        num_samples += T.inverse(torch.ones_like(maps)).sum(dim=0)
        sum_samples += T.inverse(maps).sum(dim=0)
    attention_maps = sum_samples / num_samples
    attention_maps[attention_maps != attention_maps] = 0
    return attention_maps
