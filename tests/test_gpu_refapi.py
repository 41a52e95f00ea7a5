"""The reference's own call sequence (unsupervised_keypoints/main.py:198-416, minus the
matplotlib ``visualize_attn_maps``) through the ``unsupervised_keypoints.*`` names, on the tiny
model and synthetic images.  The keyword arguments are exactly the ones the
reference passes."""
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def test_reference_main_call_sequence_through_unsupervised_keypoints(tmp_path):
    from unsupervised_keypoints.optimize_token import load_ldm
    from unsupervised_keypoints.optimize import optimize_embedding
    from unsupervised_keypoints.keypoint_regressor import find_best_indices, precompute_all_keypoints, \
        return_regressor_visible
    from unsupervised_keypoints.eval import evaluate
    from stablekeypoints_amd import _lib

    class args:   # main.py's argparse namespace at CLI-sized values
        device, model_type, feature_upsample_res = DEV, "tiny", 32
        save_folder, top_k_strategy, wandb, noise_level, lr = str(tmp_path), "gaussian", False, -1, 5e-3
        num_steps, num_tokens, layers, top_k = 2, 16, [0, 1, 2, 3], 4
        augment_degrees, augment_scale, augment_translate = 15.0, [0.8, 1.0], [0.25, 0.25]
        dataset_loc, sigma, sharpening_loss_weight, equivariance_attn_loss_weight = "~", 2.0, 100, 1000.0
        batch_size, dataset_name, max_len, furthest_point_num_samples, min_dist = 2, "synthetic", 4, 8, 0.1
        validation, num_subjects, num_indices, visualize, max_num_points = False, 1, 2, False, 2
        max_loc_strategy, augmentation_iterations, evaluation_method = "argmax", 2, "mean_average_error"

    torch.manual_seed(0)
    ldm, controllers, num_gpus = load_ldm(args.device, args.model_type, feature_upsample_res=args.feature_upsample_res)
    embedding = optimize_embedding(
        ldm, top_k_strategy=args.top_k_strategy, wandb_log=args.wandb, noise_level=args.noise_level, lr=args.lr,
        num_steps=int(args.num_steps), num_tokens=args.num_tokens, device=args.device, layers=args.layers,
        top_k=args.top_k, augment_degrees=args.augment_degrees, augment_scale=args.augment_scale,
        augment_translate=args.augment_translate, dataset_loc=args.dataset_loc, sigma=args.sigma,
        sharpening_loss_weight=args.sharpening_loss_weight,
        equivariance_attn_loss_weight=args.equivariance_attn_loss_weight, batch_size=args.batch_size,
        dataset_name=args.dataset_name, max_len=args.max_len,
        furthest_point_num_samples=args.furthest_point_num_samples, min_dist=args.min_dist,
        controllers=controllers, num_gpus=num_gpus, validation=args.validation, num_subjects=args.num_subjects)
    torch.save(embedding, os.path.join(args.save_folder, "embedding.pt"))
    assert embedding.shape == (1, 16, 32) and torch.isfinite(embedding).all()
    indices = find_best_indices(
        ldm, embedding, num_steps=args.num_indices, noise_level=args.noise_level, num_tokens=args.num_tokens,
        device=args.device, layers=args.layers, top_k=args.top_k, dataset_loc=args.dataset_loc,
        dataset_name=args.dataset_name, min_dist=args.min_dist, controllers=controllers, num_gpus=num_gpus,
        top_k_strategy=args.top_k_strategy, furthest_point_num_samples=args.furthest_point_num_samples,
        sigma=args.sigma, validation=args.validation, num_subjects=args.num_subjects)
    assert indices.dtype == torch.int64 and 1 <= indices.numel() <= args.top_k
    source_kpts, target_kpts, visible = precompute_all_keypoints(
        ldm, embedding, indices, noise_level=args.noise_level, device=args.device, layers=args.layers,
        augment_degrees=args.augment_degrees, augment_scale=args.augment_scale,
        augment_translate=args.augment_translate, augmentation_iterations=args.augmentation_iterations,
        dataset_loc=args.dataset_loc, visualize=args.visualize, dataset_name=args.dataset_name,
        controllers=controllers, num_gpus=num_gpus, max_num_points=args.max_num_points,
        max_loc_strategy=args.max_loc_strategy, save_folder=args.save_folder, validation=args.validation)
    assert source_kpts.shape == (2, indices.numel(), 2)
    if visible is None:
        visible_reshaped = torch.ones_like(target_kpts).reshape(target_kpts.shape[0], target_kpts.shape[1] * 2)
    else:
        visible_reshaped = visible.unsqueeze(-1).repeat(1, 1, 2).reshape(visible.shape[0], visible.shape[1] * 2)
    regressor = return_regressor_visible(
        source_kpts.cpu().numpy().reshape(source_kpts.shape[0], source_kpts.shape[1] * 2).astype(np.float64),
        target_kpts.cpu().numpy().reshape(target_kpts.shape[0], target_kpts.shape[1] * 2).astype(np.float64),
        visible_reshaped.cpu().numpy().astype(np.float64))
    regressor = torch.tensor(regressor).to(torch.float32)
    evaluate(ldm, embedding, indices, regressor.to(args.device), num_tokens=args.num_tokens, layers=args.layers,
             noise_level=args.noise_level, augment_degrees=args.augment_degrees, augment_scale=args.augment_scale,
             augment_translate=args.augment_translate, augmentation_iterations=args.augmentation_iterations,
             dataset_loc=args.dataset_loc, save_folder=args.save_folder, device=args.device, wandb_log=args.wandb,
             visualize=args.visualize, dataset_name=args.dataset_name, evaluation_method=args.evaluation_method,
             controllers=controllers, num_gpus=num_gpus, max_loc_strategy=args.max_loc_strategy,
             validation=args.validation)
    errs = torch.load(tmp_path / "all_errors.pt", weights_only=True)
    assert torch.isfinite(errs).all()
    # the HIP library served the whole sequence (no CPU path exists)
    assert _lib.lib() is not None
