"""CLI with the reference's flags and stages (``unsupervised_keypoints/main.py:23-416``).

optimize (``optimize_embedding`` → ``embedding.pt``) → find_indices (``find_best_indices`` →
``indices.pt``) → precompute (``precompute_all_keypoints`` → ``source_keypoints.pt``,
``target_keypoints.pt``, ``visible.pt``) → regressor (``regressor.pt``) → evaluate
(``all_errors.pt``).  ``--start_from_stage`` resumes from the saved files.  Visualisation
(``visualize_attn_maps``) is not built.  Multi-GPU: like the reference, one command uses every
visible GPU — it starts one rank per GPU under ``torch.distributed.run`` (``--num_gpus`` to pick
fewer); launching it under ``torch.distributed.run`` yourself works too (every rank seeded alike:
``--seed``).
"""
import argparse
import os
import sys

import torch


def build_parser():
    p = argparse.ArgumentParser(description="optimize a class embedding")
    p.add_argument("--model_type", type=str, default="runwayml/stable-diffusion-v1-5",
                   help="local directory of diffusers-0.8.0 UNet/VAE weights, a hub name in the local Hugging Face "
                        "cache, or 'random' / 'random-xl' / 'tiny' for seeded random weights (anything else raises)")
    p.add_argument("--dataset_loc", type=str, default="~")
    p.add_argument("--save_folder", type=str, default="outputs")
    p.add_argument("--wandb_name", type=str, default="temp")
    p.add_argument("--dataset_name", type=str, default="celeba_aligned",
                   choices=["celeba_aligned", "celeba_wild", "cub_aligned", "cub_001", "cub_002", "cub_003", "cub_all",
                            "deepfashion", "taichi", "human3.6m", "unaligned_human3.6m", "custom", "synthetic"])
    p.add_argument("--max_len", type=int, default=-1)
    p.add_argument("--start_from_stage", choices=["optimize", "find_indices", "precompute", "evaluate"],
                   default="optimize")
    p.add_argument("--device", type=str, default="cuda:0")
    p.add_argument("--wandb", action="store_true")
    p.add_argument("--lr", type=float, default=5e-3)
    p.add_argument("--num_steps", type=int, default=500)
    p.add_argument("--num_tokens", type=int, default=500)
    p.add_argument("--feature_upsample_res", type=int, default=128)
    p.add_argument("--batch_size", type=int, default=4)
    p.add_argument("--top_k_strategy", type=str, default="gaussian", choices=["entropy", "gaussian", "consistent"])
    p.add_argument("--max_loc_strategy", type=str, default="argmax", choices=["argmax", "weighted_avg"])
    p.add_argument("--evaluation_method", type=str, default="inter_eye_distance",
                   choices=["inter_eye_distance", "visible", "mean_average_error", "pck", "orientation_invariant"])
    p.add_argument("--min_dist", type=float, default=0.1)
    p.add_argument("--furthest_point_num_samples", type=int, default=25)
    p.add_argument("--num_indices", type=int, default=100)
    p.add_argument("--num_subjects", type=int, default=1)
    p.add_argument("--sharpening_loss_weight", type=float, default=100)
    p.add_argument("--equivariance_attn_loss_weight", type=float, default=1000.0)
    p.add_argument("--layers", type=int, nargs="+", default=[0, 1, 2, 3])
    p.add_argument("--noise_level", type=int, default=-1)
    p.add_argument("--max_num_points", type=int, default=50_000)
    p.add_argument("--sigma", type=float, default=2.0)
    p.add_argument("--augment_degrees", type=float, default=15.0)
    p.add_argument("--augment_scale", type=float, nargs="+", default=[0.8, 1.0])
    p.add_argument("--augment_translate", type=float, nargs="+", default=[0.25, 0.25])
    p.add_argument("--augmentation_iterations", type=int, default=10)
    p.add_argument("--visualize", action="store_true")
    p.add_argument("--validation", action="store_true")
    p.add_argument("--top_k", type=int, default=10)
    p.add_argument("--seed", type=int, default=0, help="CPU/GPU RNG seed, identical on every rank")
    p.add_argument("--num_gpus", type=int, default=-1,
                   help="ranks to start, one per GPU (-1 = every visible GPU, as the reference's DataParallel "
                        "over torch.cuda.device_count(), optimize_token.py:42-50); ignored under a launcher")
    return p


def ranks_to_start(args, visible, env):
    """How many ranks this command starts: 1 when already running as a rank (``env``) or with at
    most one GPU, else ``--num_gpus`` (every visible GPU by default)."""
    if env is not None:
        return 1
    n = visible if args.num_gpus < 0 else args.num_gpus
    if n > max(visible, 1):
        raise SystemExit(f"--num_gpus {n} but {visible} GPU(s) are visible")
    return max(n, 1)


def _load(folder, name, device=None):
    t = torch.load(os.path.join(folder, name), weights_only=True)
    return t.to(device) if (device is not None and t is not None) else t


def main(argv=None):
    import numpy as np
    args = build_parser().parse_args(argv)
    from .launch import launcher_env, spawn_ranks
    # torch.cuda.device_count() does not initialise HIP on this image, so the ranks can still start
    n = ranks_to_start(args, torch.cuda.device_count(), launcher_env())
    if n > 1:
        sys.exit(spawn_ranks(n, ["-m", "stablekeypoints_amd.main"], sys.argv[1:] if argv is None else list(argv)))
    from .eval import evaluate
    from .keypoint_regressor import (find_best_indices, precompute_all_keypoints, return_regressor,
                                     return_regressor_human36m, return_regressor_visible)
    from .optimize import optimize_embedding
    from .optimize_token import load_ldm
    if int(os.environ.get("WORLD_SIZE", "1")) > 1:
        import torch.distributed as dist
        local = int(os.environ.get("LOCAL_RANK", "0"))
        torch.cuda.set_device(local)
        args.device = f"cuda:{local}"
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    torch.manual_seed(args.seed)
    torch.cuda.manual_seed(args.seed)
    ldm, controllers, num_gpus = load_ldm(args.device, args.model_type, feature_upsample_res=args.feature_upsample_res)
    os.makedirs(args.save_folder, exist_ok=True)
    rank0 = int(os.environ.get("RANK", "0")) == 0
    stage = ["optimize", "find_indices", "precompute", "evaluate"].index(args.start_from_stage)
    common = dict(noise_level=args.noise_level, device=args.device, layers=args.layers, dataset_loc=args.dataset_loc,
                  dataset_name=args.dataset_name, controllers=controllers, num_gpus=num_gpus,
                  validation=args.validation)
    aug = dict(augment_degrees=args.augment_degrees, augment_scale=args.augment_scale,
               augment_translate=args.augment_translate)
    if stage <= 0:
        embedding = optimize_embedding(
            ldm, top_k_strategy=args.top_k_strategy, wandb_log=args.wandb, lr=args.lr, num_steps=int(args.num_steps),
            num_tokens=args.num_tokens, top_k=args.top_k, sigma=args.sigma,
            sharpening_loss_weight=args.sharpening_loss_weight,
            equivariance_attn_loss_weight=args.equivariance_attn_loss_weight, batch_size=args.batch_size,
            max_len=args.max_len, furthest_point_num_samples=args.furthest_point_num_samples, min_dist=args.min_dist,
            num_subjects=args.num_subjects, **common, **aug)
        if rank0:
            torch.save(embedding, os.path.join(args.save_folder, "embedding.pt"))
    else:
        embedding = _load(args.save_folder, "embedding.pt", args.device).detach()
    if stage <= 1:
        indices = find_best_indices(
            ldm, embedding, num_steps=args.num_indices, num_tokens=args.num_tokens, top_k=args.top_k,
            min_dist=args.min_dist, top_k_strategy=args.top_k_strategy,
            furthest_point_num_samples=args.furthest_point_num_samples, sigma=args.sigma,
            num_subjects=args.num_subjects, **common)
        if rank0:
            torch.save(indices, os.path.join(args.save_folder, "indices.pt"))
            print("indices:", indices.tolist(), flush=True)
    else:
        indices = _load(args.save_folder, "indices.pt", args.device).detach()
    if stage <= 2:
        source, target, visible = precompute_all_keypoints(
            ldm, embedding, indices, augmentation_iterations=args.augmentation_iterations,
            max_num_points=args.max_num_points, max_loc_strategy=args.max_loc_strategy,
            save_folder=args.save_folder, **common, **aug)
        if rank0:
            torch.save(source, os.path.join(args.save_folder, "source_keypoints.pt"))
            torch.save(target, os.path.join(args.save_folder, "target_keypoints.pt"))
            torch.save(visible, os.path.join(args.save_folder, "visible.pt"))
    else:
        source = _load(args.save_folder, "source_keypoints.pt", args.device)
        target = _load(args.save_folder, "target_keypoints.pt", args.device)
        visible = _load(args.save_folder, "visible.pt", args.device)
    # regressor (main.py:334-367)
    X = source.cpu().numpy().reshape(source.shape[0], -1).astype(np.float64)
    Y = target.cpu().numpy().reshape(target.shape[0], -1).astype(np.float64)
    if args.evaluation_method in ("visible", "mean_average_error"):
        if visible is None:
            vis = np.ones_like(Y)
        else:
            vis = visible.unsqueeze(-1).repeat(1, 1, 2).reshape(visible.shape[0], -1).cpu().numpy().astype(np.float64)
        regressor = return_regressor_visible(X, Y, vis)
    elif args.evaluation_method == "orientation_invariant":
        regressor = return_regressor_human36m(X, Y)
    else:
        regressor = return_regressor(X, Y)
    regressor = torch.tensor(regressor).to(torch.float32)
    if rank0:
        torch.save(regressor, os.path.join(args.save_folder, "regressor.pt"))
    evaluate(ldm, embedding, indices, regressor.to(args.device), num_tokens=args.num_tokens,
             augmentation_iterations=args.augmentation_iterations, save_folder=args.save_folder,
             evaluation_method=args.evaluation_method, max_loc_strategy=args.max_loc_strategy, **common, **aug)


if __name__ == "__main__":
    main()
