"""Token-index selection over a dataset (mirror of reference ``keypoint_regressor.find_best_indices``).

Only ``find_best_indices`` (``keypoint_regressor.py:16-121``) is on the kernels of this
package: per image a no-grad capture (``upsample_res`` bilinear maps), top-k candidates
(Gaussian KL / entropy / consistent) and furthest-point sampling, then the most frequent
token ids.  The regressor fitting and keypoint precompute stages are outside this path.
"""
import torch

from . import ptp_utils
from .datasets import make_dataset


@torch.no_grad()
def find_best_indices(ldm, context, num_steps=100, device="cuda", noise_level=-1, upsample_res=256,
                      layers=(0, 1, 2, 3, 4, 5), from_where=("down_cross", "mid_cross", "up_cross"), num_tokens=1000,
                      top_k=30, dataset_loc="~", dataset_name="celeba_aligned", min_dist=0.05,
                      furthest_point_num_samples=50, controllers=None, num_gpus=1, top_k_strategy="entropy", sigma=3,
                      validation=False, num_subjects=1, dataset=None, seed=0):
    if dataset is None:
        dataset = make_dataset(dataset_name, dataset_loc, validation=validation)
    g = torch.Generator().manual_seed(seed)
    order = torch.randperm(len(dataset), generator=g)
    indices_list = []
    for it in range(num_steps // num_gpus):
        image = dataset[int(order[it % len(order)])]["img"][None].to(device)
        attention_maps = ptp_utils.run_and_find_attn(ldm, image, context, layers=layers, noise_level=noise_level,
                                                     from_where=from_where, upsample_res=upsample_res,
                                                     controllers=controllers, device=device)
        for attention_map in attention_maps:
            if top_k_strategy == "entropy":
                cand = ptp_utils.entropy_sort(attention_map, furthest_point_num_samples)
            elif top_k_strategy == "gaussian":
                cand = ptp_utils.find_top_k_gaussian(attention_map, furthest_point_num_samples, sigma=sigma,
                                                     num_subjects=num_subjects)
            elif top_k_strategy == "consistent":
                cand = torch.arange(furthest_point_num_samples, device=attention_map.device)
            else:
                raise NotImplementedError
            indices_list.append(ptp_utils.furthest_point_sampling(attention_map, top_k, cand).cpu())
    indices_list = torch.cat(indices_list)
    import torch.distributed as dist
    if dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
        gathered = [None] * dist.get_world_size()
        dist.all_gather_object(gathered, indices_list)
        indices_list = torch.cat(gathered)
    indices, counts = torch.unique(indices_list, return_counts=True)
    indices = indices[counts.argsort(descending=True)]
    return indices[:top_k]
