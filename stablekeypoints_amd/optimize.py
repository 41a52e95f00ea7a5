"""Map aggregation, losses and the token-optimisation loop (mirror of reference ``optimize.py``).

``optimize_embedding`` keeps the reference signature (``optimize.py:269-299``).
Parallelism is one process per GPU (``torch.distributed``, RCCL over xGMI)
instead of ``nn.DataParallel``: each rank runs the reference's per-replica body on
its own image, and the token-embedding gradient is all-reduced (SUM ÷ world)
once per optimiser step, which reproduces the reference's mean over replicas
(``optimize.py:428-443``).  See DESIGN.md §Multi-GPU.
"""
import json
import time

import torch
import torch.nn.functional as F

from . import ops, ptp_utils
from . import eval as skp_eval
from .invertable_transform import RandomAffineWithInverse


def collect_maps(controller, from_where=("up_cross",), upsample_res=512, layers=(0, 1, 2, 3), indices=None):
    """optimize.py:27-79: mean over the selected stored layers and B·heads -> (N', R', R').

    Runs ``skp_aggregate`` (+ ``skp_resize_bilinear``).  As in the reference the
    upsample guard compares the token count (optimize.py:63), i.e. it fires for any
    ``upsample_res != -1``; the bilinear resize is applied after the mean, which is
    equal because both are linear.
    """
    attention_maps = controller.step_store["attn"]
    chosen = [a for li, a in enumerate(attention_maps) if li in layers]
    if not chosen:
        raise RuntimeError("collect_maps: no stored attention maps for layers %s" % (list(layers),))
    idx = None
    if indices is not None:
        idx = torch.as_tensor(indices, dtype=torch.int64)
    out = ops.aggregate(chosen, indices=idx, upsample_res=upsample_res)
    controller.reset()
    return out


def equivariance_loss(embeddings_initial, embeddings_transformed, transform, index):
    """optimize.py:157-163: mse(A, inverse(At)[index]) — only replica ``index``'s theta matters.

    ``embeddings_transformed`` is (replicas, T, h, w) or (T, h, w).
    """
    At = embeddings_transformed[index] if embeddings_transformed.dim() == 4 else embeddings_transformed
    th_inv = transform.theta_inverse()[int(index)]
    return ops.equivariance_loss_single(embeddings_initial, At, th_inv)


def sharpening_loss(attn_map, sigma=1.0, temperature=1e1, device="cuda", num_subjects=1):
    """optimize.py:166-179 (+ find_gaussian_loss_at_point 182-206): mse to Gaussians at the k-max pixels."""
    return ops.sharpening_loss(attn_map, sigma=sigma, num_subjects=num_subjects)


def find_gaussian_loss_at_point(attn_map, pos, sigma=1.0, temperature=1e-1, device="cuda", indices=None,
                                num_subjects=1):
    """optimize.py:182-206 with explicit positions pos (num, T, 2) in [0, 1]."""
    T, H, W = attn_map.shape
    target = ops.gaussian_circles(pos, H, sigma)
    if indices is not None:
        attn_map = attn_map[indices]
        target = target[indices]
    return F.mse_loss(attn_map, target)


def _make_dataset(dataset_name, dataset_loc, max_len, validation):
    from . import datasets
    return datasets.make_dataset(dataset_name, dataset_loc, max_len=max_len, validation=validation)


def _world():
    import torch.distributed as dist
    if dist.is_available() and dist.is_initialized():
        return dist.get_world_size(), dist.get_rank()
    return 1, 0


def optimize_embedding(ldm, top_k_strategy="entropy", wandb_log=True, context=None, device="cuda", num_steps=2000,
                       from_where=("down_cross", "mid_cross", "up_cross"), upsample_res=256, layers=(0, 1, 2, 3, 4, 5),
                       lr=5e-3, noise_level=-1, num_tokens=1000, top_k=10, augment_degrees=30,
                       augment_scale=(0.9, 1.1), augment_translate=(0.1, 0.1), dataset_loc="~", sigma=1.0,
                       sharpening_loss_weight=100, equivariance_attn_loss_weight=100, batch_size=4, num_gpus=1,
                       dataset_name="celeba_aligned", max_len=-1, min_dist=0.05, furthest_point_num_samples=50,
                       controllers=None, validation=False, num_subjects=1, dataset=None, log=None, seed=None,
                       step_callback=None):
    """optimize.py:269-475.  Extra keyword-only conveniences: ``dataset`` (an object
    yielding {"img": (3,H,W)}; overrides dataset_name), ``log`` (callable receiving
    the per-step metrics dict instead of wandb/print), ``seed`` (per-rank sampler
    seed), ``step_callback(iteration)`` (called after every micro-iteration)."""
    world, rank = _world()
    if num_gpus != world:
        num_gpus = world   # one process per GPU: the replica count is the world size
    if dataset is None:
        dataset = _make_dataset(dataset_name, dataset_loc, max_len, validation)
    invertible_transform = RandomAffineWithInverse(degrees=augment_degrees, scale=augment_scale,
                                                   translate=augment_translate)
    if context is None:
        context = ptp_utils.init_random_noise(device, num_words=num_tokens)
    context.requires_grad = True
    optimizer = torch.optim.Adam([context], lr=lr)

    accum = batch_size // num_gpus
    n_iter = int(num_steps * accum)
    gen = torch.Generator().manual_seed(seed if seed is not None else torch.initial_seed() % (2 ** 31))
    sampler_gen = torch.Generator().manual_seed(int(torch.randint(0, 2 ** 31 - 1, (1,), generator=gen)) + rank)
    order = torch.randperm(len(dataset), generator=sampler_gen)
    pos = 0

    start = time.time()
    it_start = time.time()
    run_eq = run_sh = run_tot = 0.0
    for iteration in range(n_iter):
        if pos >= len(order):
            order = torch.randperm(len(dataset), generator=sampler_gen)
            pos = 0
        image = dataset[int(order[pos])]["img"][None].to(device, non_blocking=True)
        pos += 1

        kw = dict(layers=layers, noise_level=noise_level, from_where=from_where, upsample_res=-1, device=device,
                  controllers=controllers)
        attn_maps = ptp_utils.run_and_find_attn(ldm, image, context, **kw)
        transformed_img = invertible_transform(image)
        attention_maps_transformed = ptp_utils.run_and_find_attn(ldm, transformed_img, context, **kw)

        attn_map, attention_map_transformed = attn_maps[0], attention_maps_transformed[0]
        if top_k_strategy == "entropy":
            top_embedding_indices = ptp_utils.entropy_sort(attn_map, furthest_point_num_samples)
        elif top_k_strategy == "gaussian":
            top_embedding_indices = ptp_utils.find_top_k_gaussian(attn_map, furthest_point_num_samples, sigma=sigma,
                                                                  num_subjects=num_subjects)
        elif top_k_strategy == "consistent":
            top_embedding_indices = torch.arange(furthest_point_num_samples, device=attn_map.device)
        else:
            raise NotImplementedError
        top_embedding_indices = ptp_utils.furthest_point_sampling(attention_map_transformed, top_k,
                                                                  top_embedding_indices)
        _sharpening_loss = sharpening_loss(attn_map[top_embedding_indices], device=device, sigma=sigma,
                                           num_subjects=num_subjects)
        _loss_equivariance_attn = equivariance_loss(attn_map[top_embedding_indices],
                                                    attention_map_transformed[top_embedding_indices][None],
                                                    invertible_transform, 0)

        loss = _loss_equivariance_attn * equivariance_attn_loss_weight + _sharpening_loss * sharpening_loss_weight
        run_eq = run_eq + _loss_equivariance_attn.detach() / accum * equivariance_attn_loss_weight
        run_sh = run_sh + _sharpening_loss.detach() / accum * sharpening_loss_weight
        run_tot = run_tot + loss.detach() / accum
        loss = loss / accum
        loss.backward()
        if step_callback is not None:
            step_callback(iteration)

        if (iteration + 1) % accum == 0:
            if world > 1:
                import torch.distributed as dist
                dist.all_reduce(context.grad, op=dist.ReduceOp.SUM)
                context.grad.div_(world)
                stats = torch.stack([run_tot, run_eq, run_sh])
                dist.all_reduce(stats, op=dist.ReduceOp.SUM)
                run_tot, run_eq, run_sh = (stats / world).unbind(0)
            optimizer.step()
            optimizer.zero_grad()
            rec = {"loss": float(run_tot), "running_equivariance_attn_loss": float(run_eq),
                   "running_sharpening_loss": float(run_sh), "iteration time": time.time() - it_start}
            if log is not None:
                log(rec)
            elif rank == 0 and wandb_log:
                print(json.dumps(rec), flush=True)
            elif rank == 0:
                print(f"loss: {rec['loss']}, _loss_equivariance_attn: {rec['running_equivariance_attn_loss']} "
                      f"sharpening_loss: {rec['running_sharpening_loss']}, iteration time: {rec['iteration time']}",
                      flush=True)
            run_eq = run_sh = run_tot = 0.0
            it_start = time.time()
    if rank == 0 and log is None:
        print(f"optimization took {time.time() - start} seconds", flush=True)
    return context.detach()
