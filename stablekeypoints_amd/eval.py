"""Keypoint extraction: argmax / soft-argmax and test-time augmentation (mirror of reference ``eval.py``).

``find_max_pixel``, ``find_k_max_pixels``, ``mask_radius`` and
``pixel_from_weighted_avg`` (``eval.py:39-155``) run as HIP kernels with the
reference's semantics (first-occurrence argmax, NaN is max, in-place mutation in
``pixel_from_weighted_avg``).  ``run_image_with_context_augmented`` (``:197-355``) is the
test-time-augmentation average on the same kernels; ``evaluate`` (``:374-539``) regresses
keypoints from it and scores them with the reference's five metrics (``keypoint_error``).
"""
import os

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


# default TTA batch bound: warped copies per capture pass × pixels per copy (10 copies at 512², the
# measured TTA setting, profiles/r03ao_bench_tta.json)
AUG_BATCH_PIXELS = 10 * 512 * 512


@torch.no_grad()
def run_image_with_context_augmented(ldm, image, context, indices, device="cuda",
                                     from_where=("down_cross", "mid_cross", "up_cross"), layers=(0, 1, 2, 3, 4, 5),
                                     augmentation_iterations=20, noise_level=-1, augment_degrees=30,
                                     augment_scale=(0.9, 1.1), augment_translate=(0.1, 0.1), visualize=False,
                                     controllers=None, num_gpus=1, save_folder="outputs", upscale_size=512,
                                     augmentation_batch=None):
    """eval.py:197-355 (hot part 221-266, 327-330): TTA-averaged maps of the chosen tokens.

    ``image`` is (3, H, W) in [0, 1] (torch or numpy HWC).  Each of the
    ``augmentation_iterations // num_gpus`` iterations draws ``num_gpus`` thetas from the CPU
    generator in the reference's order (one per replica, eval.py:238-242).  Replica r's warped
    copy is captured (``indices`` gathered, bilinear to ``upscale_size``: collect_maps), then its
    map and a ones map are inverse-warped and summed.  Returns Σmaps / Σones with NaN → 0.

    ``augmentation_batch`` (extra; None = as many iterations as ``AUG_BATCH_PIXELS`` allows: 10
    at 512², 2 at SDXL's 1024²): how many iterations' warped copies go through ONE batched
    VAE/UNet capture pass.  Peak activation memory grows linearly with it (the reference's loop
    holds one copy at a time), so the default is bounded by image area.  Every copy is captured on its
    own (per-image maps, ``run_and_find_attn_per_image``), the thetas are drawn iteration by
    iteration exactly as the reference draws them, and the copies' contributions are summed in
    iteration order, so this is the reference's loop up to fp32 summation order and the GPU
    noise draw (one ``randn_like`` per batch instead of per copy; the reference's CUDA noise is
    not reproducible on another device anyway).  At batch 1 a 64² latent UNet pass cannot fill
    256 CUs; 10 copies in one pass do.

    Replicas: with torch.distributed initialised and ``num_gpus`` equal to the world size,
    rank r runs replica r of every iteration and the two (n, S, S) sums are all-reduced (SUM)
    once at the end; every rank must hold the same CPU RNG state (same seed) so that all draw
    the same thetas.  In one process, the ``num_gpus`` copies of an iteration are captured in
    the same batched pass.
    """
    if visualize:
        raise NotImplementedError("visualisation is outside the hot path")
    from .optimize import _world
    img = image if torch.is_tensor(image) else torch.as_tensor(image)
    if img.dim() == 3 and img.shape[-1] == 3 and img.shape[0] != 3:
        img = img.permute(2, 0, 1)
    img = img.to(device, torch.float32)
    world, rank = _world()
    if world > 1 and num_gpus != world:
        raise ValueError(f"num_gpus={num_gpus} must equal the world size {world} (one replica per rank)")
    n = len(indices)
    num_samples = torch.zeros(n, upscale_size, upscale_size, device=device)
    sum_samples = torch.zeros(n, upscale_size, upscale_size, device=device)
    T = RandomAffineWithInverse(degrees=augment_degrees, scale=augment_scale, translate=augment_translate)
    iters = augmentation_iterations // num_gpus
    if augmentation_batch is None:
        augmentation_batch = max(1, AUG_BATCH_PIXELS // (img.shape[-1] * img.shape[-2] * max(1, num_gpus // world)))
    chunk = max(1, int(augmentation_batch))
    done = 0
    while done < iters:
        c = min(chunk, iters - done)
        # every rank draws all replicas' thetas, iteration by iteration (eval.py:238-242)
        theta = torch.cat([T.draw_theta(num_gpus) for _ in range(c)])
        if world > 1:
            theta = theta.reshape(c, num_gpus, 2, 3)[:, rank]
        aug = T(img[None].expand(theta.shape[0], -1, -1, -1), theta=theta)
        if aug.shape[0] == 1:
            maps = torch.stack(ptp_utils.run_and_find_attn(
                ldm, aug, context, layers=layers, noise_level=noise_level, from_where=from_where,
                upsample_res=upscale_size, device=device, controllers=controllers, indices=indices))
        else:
            per = ptp_utils.run_and_find_attn_per_image(ldm, aug, context, noise_level=noise_level, device=device,
                                                        layers=layers, upsample_res=upscale_size, indices=indices,
                                                        controllers=controllers)
            maps = torch.stack([per[k][b] for b in range(aug.shape[0]) for k in range(len(per))])
        num_samples += T.inverse(torch.ones_like(maps)).sum(dim=0)
        sum_samples += T.inverse(maps).sum(dim=0)
        done += c
    if world > 1:
        import torch.distributed as dist
        dist.all_reduce(num_samples)
        dist.all_reduce(sum_samples)
    attention_maps = sum_samples / num_samples
    attention_maps[attention_maps != attention_maps] = 0
    return attention_maps


def swap_points(points):
    """eval.py:358-370: left/right keypoint permutation of Human3.6M (B, K, D)."""
    pairs = [(1, 6), (2, 7), (3, 8), (4, 9), (5, 10), (17, 25), (18, 26), (19, 27), (20, 28), (21, 28), (22, 30),
             (23, 31)]
    perm = list(range(points.shape[1]))
    for a, b in pairs:
        perm[a], perm[b] = b, a
    return points[:, perm, :]


METRICS = ("inter_eye_distance", "visible", "mean_average_error", "pck", "orientation_invariant")


def keypoint_error(highest_indices, regressor, gt_kpts, evaluation_method="inter_eye_distance", visible=None):
    """One image's error (eval.py:467-513): regress (row, col)/512 maxima of the chosen tokens
    to keypoints, ``((p − 0.5) @ W) + 0.5``, and score them against ``gt_kpts`` (K, 2).

    inter_eye_distance: mean L2 / |gt₀ − gt₁|; visible: Σ L2·v / Σ v; mean_average_error:
    Σ L2·v at 256 px scale; pck: fraction within 6 px at 256 px scale; orientation_invariant:
    min over the left/right swap of the mean L2, × 128.
    """
    if evaluation_method not in METRICS:
        raise ValueError(f"evaluation_method must be one of {METRICS}")
    est = ((highest_indices.reshape(1, -1) - 0.5) @ regressor) + 0.5
    est = est.reshape(-1, 2)
    gt = gt_kpts.to(est.device, est.dtype)
    if evaluation_method in ("mean_average_error", "pck"):
        est = est * 256
        gt = gt * 256
    l2 = (est - gt).norm(dim=-1)
    if evaluation_method == "inter_eye_distance":
        eye = torch.sqrt(torch.sum((gt[0] - gt[1]) ** 2, dim=-1))
        return torch.mean(l2 / eye)
    if evaluation_method in ("visible", "mean_average_error"):
        vis = torch.ones_like(l2) if visible is None else visible.to(l2.device, l2.dtype)
        err = (l2 * vis).sum()
        return err / vis.sum() if evaluation_method == "visible" else err
    if evaluation_method == "pck":
        return (l2 < 6).float().mean()
    err = l2.mean()
    swapped = (swap_points(est[None])[0] - gt).norm(dim=-1).mean()
    return torch.minimum(err, swapped) * 128


@torch.no_grad()
def evaluate(ldm, context, indices, regressor, device="cuda", from_where=("down_cross", "mid_cross", "up_cross"),
             upsample_res=32, layers=(0, 1, 2, 3, 4, 5), noise_level=-1, num_tokens=1000, augment_degrees=30,
             augment_scale=(0.9, 1.1), augment_translate=(0.1, 0.1), augmentation_iterations=20, dataset_loc="~",
             save_folder="outputs", wandb_log=False, visualize=False, dataset_name="celeba_aligned",
             evaluation_method="inter_eye_distance", controllers=None, num_gpus=1, max_loc_strategy="argmax",
             validation=False, dataset=None, upscale_size=512):
    """eval.py:374-539: per test image (shuffled loader, batch 1) the TTA maps of ``indices``,
    their maxima / 512, the regressed keypoints and ``keypoint_error``; writes
    ``all_errors.pt`` (per-image errors) to ``save_folder`` and returns the mean error.
    ``dataset`` (extra) overrides the lookup; ``visualize``/``wandb_log`` are not supported.
    """
    from .datasets import make_dataset
    if evaluation_method not in METRICS:
        raise ValueError(f"evaluation_method must be one of {METRICS}")
    if dataset is None:
        dataset = make_dataset(dataset_name, dataset_loc, validation=validation, split="test")
    loader = torch.utils.data.DataLoader(dataset, batch_size=1, shuffle=True, drop_last=True)
    it = iter(loader)
    regressor = regressor.to(device, torch.float32)
    values = []
    for _ in range(len(dataset)):
        batch = next(it)
        maps = run_image_with_context_augmented(
            ldm, batch["img"][0], context, indices.cpu(), device=device, from_where=from_where, layers=layers,
            noise_level=noise_level, augmentation_iterations=augmentation_iterations, augment_degrees=augment_degrees,
            augment_scale=augment_scale, augment_translate=augment_translate, controllers=controllers,
            num_gpus=num_gpus, save_folder=save_folder, upscale_size=upscale_size)
        if max_loc_strategy == "argmax":
            highest = find_max_pixel(maps) / 512.0
        else:
            highest = pixel_from_weighted_avg(maps) / 512.0
        vis = batch["visibility"][0] if "visibility" in batch else None
        values.append(float(keypoint_error(highest, regressor, batch["kpts"][0], evaluation_method, vis)))
    os.makedirs(save_folder, exist_ok=True)
    torch.save(torch.tensor(values), os.path.join(save_folder, "all_errors.pt"))
    mean = float(torch.tensor(values).mean()) if values else float("nan")
    print(f"mean distance: {mean}", flush=True)
    return mean
