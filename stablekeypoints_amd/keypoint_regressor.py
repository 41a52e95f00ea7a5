"""Token-index selection and keypoint precompute over a dataset (mirror of reference
``keypoint_regressor.py``).

``find_best_indices`` (``keypoint_regressor.py:16-121``): per image a no-grad capture
(``upsample_res`` bilinear maps), top-k candidates (Gaussian KL / entropy / consistent) and
furthest-point sampling on the HIP kernels, then the most frequent token ids.
``precompute_all_keypoints`` (``:124-224``): per image the TTA-averaged maps of the chosen
tokens (``eval.run_image_with_context_augmented``) and their argmax / soft-argmax / 512.
``return_regressor`` / ``return_regressor_visible`` / ``return_regressor_human36m``
(``:227-299``): the least-squares keypoint regressor (host numpy/torch, as in the reference).

Multi-GPU: one process per GPU.  The reference's ``num_gpus`` DataParallel replicas become
ranks: the data order is drawn once (CPU generator; every rank must be seeded alike) and rank
r takes replica r's image of every batch (find_best_indices, then an all_gather of the index
lists) or replica r's augmentations of every image (precompute, via the TTA all-reduce).
"""
import numpy as np
import torch

from . import ptp_utils
from .datasets import make_dataset
from .eval import find_max_pixel, pixel_from_weighted_avg, run_image_with_context_augmented


def _loader(dataset, batch_size):
    """DataLoader(shuffle=True, drop_last=True) as the reference builds it.  Its shuffle seed
    comes from the CPU generator, so ranks seeded alike draw the same order (no collective)."""
    return torch.utils.data.DataLoader(dataset, batch_size=batch_size, shuffle=True, drop_last=True)


def _next(state):
    try:
        return next(state["it"])
    except StopIteration:   # keypoint_regressor.py:76-80: restart the loader
        state["it"] = iter(state["loader"])
        return next(state["it"])


@torch.no_grad()
def find_best_indices(ldm, context, num_steps=100, device="cuda", noise_level=-1, upsample_res=256,
                      layers=(0, 1, 2, 3, 4, 5), from_where=("down_cross", "mid_cross", "up_cross"), num_tokens=1000,
                      top_k=30, dataset_loc="~", dataset_name="celeba_aligned", min_dist=0.05,
                      furthest_point_num_samples=50, controllers=None, num_gpus=1, top_k_strategy="entropy", sigma=3,
                      validation=False, num_subjects=1, dataset=None, capture_batch=8):
    """keypoint_regressor.py:16-121.  ``dataset`` (extra) overrides the dataset_name lookup.

    ``capture_batch`` (extra): how many of this rank's images go through ONE batched VAE/UNet
    capture pass (``run_and_find_attn_per_image``: maps per image, exactly what one
    ``run_and_find_attn`` per image gives, up to the GPU noise draw — one ``randn_like`` per
    batch).  The images are taken from the loader in the reference's order and their
    candidates / FPS picks appended in that order, so the ranking is the reference's.  1 = the
    reference's one pass per image."""
    from .optimize import _world
    if top_k_strategy not in ("entropy", "gaussian", "consistent"):
        raise NotImplementedError(top_k_strategy)
    if dataset is None:
        dataset = make_dataset(dataset_name, dataset_loc, validation=validation)
    world, rank = _world()
    if world > 1 and num_gpus != world:
        raise ValueError(f"num_gpus={num_gpus} must equal the world size {world} (one replica per rank)")
    loader = _loader(dataset, num_gpus)
    state = {"loader": loader, "it": iter(loader)}
    indices_list = []
    steps = num_steps // num_gpus
    chunk = max(1, int(capture_batch))

    def load(c):
        """The next c loader batches, this rank's replica of each (the reference's per-device
        image), on the device via pinned memory without waiting for the queued GPU work."""
        groups = [_next(state)["img"] for _ in range(c)]
        mine = torch.cat([g[rank:rank + 1] if world > 1 else g for g in groups])
        if torch.device(device).type == "cuda" and mine.device.type == "cpu":
            return mine.pin_memory().to(device, non_blocking=True)
        return mine.to(device)   # a dataset that yields device tensors (or a CPU run)

    done = 0
    nxt = load(min(chunk, steps)) if steps > 0 else None
    while done < steps:
        c = min(chunk, steps - done)
        mine = nxt
        if mine.shape[0] == 1:
            per_image = [ptp_utils.run_and_find_attn(ldm, mine, context, layers=layers, noise_level=noise_level,
                                                     from_where=from_where, upsample_res=upsample_res,
                                                     controllers=controllers, device=device)]
        else:
            per = ptp_utils.run_and_find_attn_per_image(ldm, mine, context, noise_level=noise_level, device=device,
                                                        layers=layers, upsample_res=upsample_res,
                                                        controllers=controllers, stacked=True)
            if all(torch.is_tensor(p) for p in per) and _select_batched(top_k_strategy, top_k,
                                                                         furthest_point_num_samples):
                # image b's maps (in the reference's per-device order) in one (B', N, S, S) stack
                stack = per[0] if len(per) == 1 else torch.stack(
                    [p[b] for b in range(mine.shape[0]) for p in per])
                sel, n = _select_stack(stack, top_k, furthest_point_num_samples, top_k_strategy, sigma,
                                       num_subjects)
                # the next batch is drawn and uploaded while this one's kernels run; then the picks
                # come back (the loader's draws keep the reference's order)
                nxt = load(min(chunk, steps - done - c)) if done + c < steps else None
                sel, n = sel.cpu(), n.cpu()
                indices_list.extend(sel[b, :int(n[b])] for b in range(sel.shape[0]))
                done += c
                continue
            per_image = [[per[k][b] for k in range(len(per))] for b in range(mine.shape[0])]
        for attention_maps in per_image:
            for attention_map in attention_maps:
                if top_k_strategy == "entropy":
                    cand = ptp_utils.entropy_sort(attention_map, furthest_point_num_samples)
                elif top_k_strategy == "gaussian":
                    cand = ptp_utils.find_top_k_gaussian(attention_map, furthest_point_num_samples, sigma=sigma,
                                                         num_subjects=num_subjects)
                else:
                    cand = torch.arange(furthest_point_num_samples, device=attention_map.device)
                indices_list.append(ptp_utils.furthest_point_sampling(attention_map, top_k, cand).cpu())
        done += c
        if done < steps:
            nxt = load(min(chunk, steps - done))
    indices_list = torch.cat(indices_list)
    if world > 1:
        import torch.distributed as dist
        gathered = [None] * world
        dist.all_gather_object(gathered, indices_list)
        indices_list = torch.cat(gathered)
    indices, counts = torch.unique(indices_list, return_counts=True)
    indices = indices[counts.argsort(descending=True)]
    return indices[:top_k]


def _select_batched(strategy, top_k, n_cand):
    """The one-launch-per-stage selection applies: a batched candidate ranking exists for the
    strategy and the FPS kernel's bounds hold (top_k ≥ 2 picks from ≥ 2 candidates)."""
    return strategy in ("gaussian", "entropy", "consistent") and top_k >= 2 and n_cand >= 2


def _select_stack(stack, top_k, n_cand, strategy, sigma, num_subjects):
    """The reference's per-image candidates + furthest-point sampling (keypoint_regressor.py:95-112)
    for every image of a (B, N, S, S) stack: the keys of every row in one launch (the Gaussian KL, or
    the entropies for the entropy strategy), the ranking + the candidates' argmax in one, FPS in one
    (consistent: an arange and skp_fps_batch).  Returns the device tensors ((B, top_k) picks, (B,)
    counts): image b's picks are the first counts[b] (fewer when its FPS ran out of candidates, as
    the reference's list, ptp_utils.py:156-157)."""
    from . import ops
    B, N = stack.shape[:2]
    if strategy == "gaussian":    # KL keys → ranking + the candidates' argmax → FPS: 3 launches
        return ops.gaussian_fps_batch(stack, stack, n_cand, top_k, sigma=sigma, num_subjects=num_subjects)[:2]
    if strategy == "entropy":     # keypoint_regressor.py:104-105: entropy keys → ranking + argmax → FPS
        return ops.fps_from_keys_batch(ops.entropy_keys_batch(stack), stack, n_cand, top_k)[:2]
    cand = torch.arange(n_cand, device=stack.device).expand(B, n_cand)
    return ops.furthest_point_sampling_batch(stack, top_k, cand)


@torch.no_grad()
def precompute_all_keypoints(ldm, context, top_indices, device="cuda", noise_level=-1, layers=(0, 1, 2, 3, 4, 5),
                             from_where=("down_cross", "mid_cross", "up_cross"), augment_degrees=30,
                             augment_scale=(0.9, 1.1), augment_translate=(0.1, 0.1), augmentation_iterations=20,
                             dataset_loc="~", visualize=False, dataset_name="celeba_aligned", controllers=None,
                             num_gpus=1, max_num_points=50_000, max_loc_strategy="argmax", save_folder="outputs",
                             validation=False, dataset=None, upscale_size=512):
    """keypoint_regressor.py:124-224: (source (P, n, 2), target (P, K, 2), visibility (P, K) or None).

    ``dataset`` (extra) overrides the lookup; its items need "img" and "kpts" (and optionally
    "visibility"), like the reference's *RegSet readers.
    """
    if dataset is None:
        dataset = make_dataset(dataset_name, dataset_loc, validation=validation)
    loader = _loader(dataset, 1)
    it = iter(loader)
    source, target, visibility = [], [], []
    for _ in range(min(len(dataset), max_num_points)):
        mb = next(it)
        target.append(mb["kpts"][0])
        if "visibility" in mb:
            visibility.append(mb["visibility"][0])
        maps = run_image_with_context_augmented(
            ldm, mb["img"][0], context, top_indices, device=device, from_where=from_where, layers=layers,
            noise_level=noise_level, augmentation_iterations=augmentation_iterations, augment_degrees=augment_degrees,
            augment_scale=augment_scale, augment_translate=augment_translate, controllers=controllers,
            save_folder=save_folder, num_gpus=num_gpus, upscale_size=upscale_size)
        if max_loc_strategy == "argmax":
            source.append(find_max_pixel(maps) / 512.0)
        else:
            source.append(pixel_from_weighted_avg(maps) / 512.0)
    return torch.stack(source), torch.stack(target), (torch.stack(visibility) if visibility else None)


def return_regressor(X, Y):
    """keypoint_regressor.py:246-256: W = pinv(XᵀX) Xᵀ Y on centred coordinates."""
    X = np.asarray(X) - 0.5
    Y = np.asarray(Y) - 0.5
    return np.linalg.pinv(X.T @ X) @ X.T @ Y


def return_regressor_visible(X, Y, visible):
    """keypoint_regressor.py:227-243: one least-squares column per keypoint over the images
    where that keypoint is visible."""
    X = np.asarray(X) - 0.5
    Y = np.asarray(Y) - 0.5
    visible = np.asarray(visible)
    W = np.zeros((X.shape[1], Y.shape[1]))
    for j in range(Y.shape[1]):
        rows = np.where(visible[:, j] == 1)[0]
        Xj = X[rows, :]
        W[:, j] = np.linalg.pinv(Xj.T @ Xj) @ Xj.T @ Y[rows, j]
    return W


def return_regressor_human36m(X, Y):
    """keypoint_regressor.py:266-299: least squares with left/right label swaps — while more
    than 10 images sit closer to their swapped labels, swap those and refit."""
    from .eval import swap_points
    X = torch.as_tensor(X) - 0.5
    Y = torch.as_tensor(Y) - 0.5
    XTXXT = (X.T @ X).inverse() @ X.T
    while True:
        W = XTXXT @ Y
        pred = X @ W
        dist = (pred - Y).reshape(X.shape[0], -1, 2).norm(dim=2).mean(dim=1)
        swapped = swap_points(Y.reshape(Y.shape[0], -1, 2)).reshape(Y.shape[0], -1)
        swapped_dist = (pred - swapped).reshape(X.shape[0], -1, 2).norm(dim=2).mean(dim=1)
        should = dist > swapped_dist
        if should.sum() > 10:
            Y[should] = swapped[should]
        else:
            break
    return W.numpy()
