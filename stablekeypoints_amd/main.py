"""CLI with the reference's flags (``unsupervised_keypoints/main.py:23-196``).

Stages on this package's path: ``optimize`` (``optimize_embedding`` → ``embedding.pt``) and
``find_indices`` (``find_best_indices`` → ``indices.pt``).  The later stages (keypoint
precompute, regressor fitting, visualisation, evaluation) are outside the MI355X hot path.
Multi-GPU: ``python -m torch.distributed.run --nproc-per-node N -m stablekeypoints_amd.main ...``.
"""
import argparse
import os

import torch


def build_parser():
    p = argparse.ArgumentParser(description="optimize a class embedding")
    p.add_argument("--model_type", type=str, default="runwayml/stable-diffusion-v1-5",
                   help="local directory of diffusers-0.8.0 UNet/VAE weights; other values: seeded random SD-1.5")
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
    return p


def main(argv=None):
    args = build_parser().parse_args(argv)
    from .optimize import optimize_embedding
    from .optimize_token import load_ldm
    from .keypoint_regressor import find_best_indices
    if int(os.environ.get("WORLD_SIZE", "1")) > 1:
        import torch.distributed as dist
        local = int(os.environ.get("LOCAL_RANK", "0"))
        torch.cuda.set_device(local)
        args.device = f"cuda:{local}"
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    ldm, controllers, num_gpus = load_ldm(args.device, args.model_type, feature_upsample_res=args.feature_upsample_res)
    os.makedirs(args.save_folder, exist_ok=True)
    rank0 = int(os.environ.get("RANK", "0")) == 0
    if args.start_from_stage == "optimize":
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
        if rank0:
            torch.save(embedding, os.path.join(args.save_folder, "embedding.pt"))
    else:
        embedding = torch.load(os.path.join(args.save_folder, "embedding.pt"), weights_only=True).to(args.device)
    if args.start_from_stage in ("optimize", "find_indices"):
        indices = find_best_indices(
            ldm, embedding, num_steps=args.num_indices, noise_level=args.noise_level, num_tokens=args.num_tokens,
            device=args.device, layers=args.layers, top_k=args.top_k, dataset_loc=args.dataset_loc,
            dataset_name=args.dataset_name, min_dist=args.min_dist, controllers=controllers, num_gpus=num_gpus,
            top_k_strategy=args.top_k_strategy, furthest_point_num_samples=args.furthest_point_num_samples,
            sigma=args.sigma, validation=args.validation, num_subjects=args.num_subjects)
        if rank0:
            torch.save(indices, os.path.join(args.save_folder, "indices.pt"))
            print("indices:", indices.tolist(), flush=True)
    if args.start_from_stage in ("precompute", "evaluate"):
        raise SystemExit("stages 'precompute'/'evaluate' (regressor, metrics) are outside the MI355X hot path")


if __name__ == "__main__":
    main()
