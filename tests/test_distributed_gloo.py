"""Multi-rank semantics of the token optimisation on CPU (gloo, world_size 2).

The reference runs one replica per GPU under nn.DataParallel and averages the per-replica
losses (optimize.py:428-443).  Here each rank is a process; TokenOptimizer all-reduces the
context gradient (SUM ÷ world) once per optimiser step.  These tests check that sharding the
images over 2 ranks gives the same gradient, loss statistics and Adam update as one rank
processing all of them, using a CPU surrogate for the per-image loss (the real per-image loss
runs on HIP kernels and is covered by tests/test_gpu_parity.py).
"""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _make_opt(context, accum):
    from stablekeypoints_amd.optimize import TokenOptimizer

    class Surrogate(TokenOptimizer):
        def __init__(self, context, accum):   # no model: the loss is a CPU surrogate
            self.context = context
            self.context.requires_grad = True
            self.optimizer = torch.optim.Adam([self.context], lr=5e-3)
            self.accum, self.w_eq, self.w_sharp = accum, 1000.0, 100.0
            self.batch_captures = False
            self.world = dist.get_world_size() if dist.is_initialized() else 1
            self.reset_running()

        def image_loss(self, image):
            w = image.flatten()[: self.context.numel()].reshape(self.context.shape)
            eq = ((self.context - w) ** 2).mean()
            sh = (self.context * w).sum().abs() / w.numel()
            return eq * self.w_eq + sh * self.w_sharp, eq, sh, None
    return Surrogate(context, accum)


def _images(n):
    g = torch.Generator().manual_seed(7)
    return [torch.rand(1, 3, 8, 8, generator=g) * 2 for _ in range(n)]


def _reference_single(n_img, steps):
    ctx = torch.randn(1, 4, 6, generator=torch.Generator().manual_seed(3))
    opt = _make_opt(ctx, n_img)
    imgs = _images(n_img * steps)
    recs, grads = [], []
    for st in range(steps):
        for i in range(n_img):
            opt.micro_step(imgs[st * n_img + i])
        grads.append(opt.context.grad.clone())
        recs.append({k: float(v) for k, v in opt.optimizer_step().items()})
    return opt.context.detach().clone(), recs, grads


def _worker(rank, world, port, n_img, steps, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        ctx = torch.randn(1, 4, 6, generator=torch.Generator().manual_seed(3))
        per_rank = n_img // world
        opt = _make_opt(ctx, per_rank)
        imgs = _images(n_img * steps)
        recs = []
        for st in range(steps):
            for i in range(per_rank):   # rank r takes images r*per_rank ... of each global batch
                opt.micro_step(imgs[st * n_img + rank * per_rank + i])
            recs.append({k: float(v) for k, v in opt.optimizer_step().items()})
        q.put((rank, opt.context.detach().numpy().copy(), recs))   # by value: no fd sharing
    finally:
        dist.destroy_process_group()


def test_two_rank_grad_allreduce_equals_single_rank():
    n_img, steps, world = 4, 3, 2
    ref_ctx, ref_recs, _ = _reference_single(n_img, steps)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, n_img, steps, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, c, recs in out:
        c = torch.from_numpy(c)
        assert torch.allclose(c, ref_ctx, atol=1e-6, rtol=1e-5), f"rank {rank} context diverged"
        for a, b in zip(recs, ref_recs):
            for k in a:
                assert abs(a[k] - b[k]) <= 1e-5 * max(1.0, abs(b[k])), (k, a[k], b[k])


# ---------------------------------------------------------------------------- eval-side stages
# find_best_indices / run_image_with_context_augmented on 2 ranks == one process running the
# reference's num_gpus=2 replicas.  The capture, selection and warp ops are HIP kernels; here
# they are replaced by CPU stand-ins that depend on the image content and theta, so the test
# checks the replica ↔ rank mapping, the shared shuffle / theta draws and the collectives.
def _stub_eval_stages(monkeypatch_like):
    from stablekeypoints_amd import ptp_utils
    from stablekeypoints_amd.invertable_transform import RandomAffineWithInverse

    def fake_maps(image, indices=None):
        img = image.reshape(image.shape[0], -1)
        base = torch.arange(16.0).reshape(16, 1, 1) * 0.01
        maps = base + img.mean(dim=1).reshape(-1, 1, 1, 1)[0] * torch.linspace(0, 1, 64).reshape(1, 8, 8)
        maps = maps * (1 + torch.arange(16.0).reshape(16, 1, 1) * img[0, 0])
        return maps if indices is None else maps[torch.as_tensor(indices)]

    def run_and_find_attn(ldm, image, context, indices=None, **kw):
        return [fake_maps(image, indices)]

    def run_and_find_attn_per_image(ldm, images, context, indices=None, **kw):
        return [[fake_maps(images[b:b + 1], indices) for b in range(images.shape[0])]]

    def topk(maps, k, **kw):
        return torch.argsort(maps.reshape(maps.shape[0], -1).sum(1), descending=True)[:k]

    def fps(maps, k, cand):
        return torch.as_tensor(cand)[[0, len(cand) - 1]][:k]

    def warp(self, img, theta=None):
        if theta is None:
            theta = self.draw_theta(img.shape[0])
        self.last_params = {"theta": theta}
        return img * theta[:, 0, 0].reshape(-1, 1, 1, 1) + theta[:, 0, 2].reshape(-1, 1, 1, 1)

    def inverse(self, x):
        th = self.last_params["theta"]
        return (x - th[:, 0, 2].reshape(-1, 1, 1, 1)) * th[:, 1, 1].reshape(-1, 1, 1, 1)

    for obj, name, fn in [(ptp_utils, "run_and_find_attn", run_and_find_attn),
                          (ptp_utils, "run_and_find_attn_per_image", run_and_find_attn_per_image),
                          (ptp_utils, "find_top_k_gaussian", topk), (ptp_utils, "entropy_sort", topk),
                          (ptp_utils, "furthest_point_sampling", fps),
                          (RandomAffineWithInverse, "__call__", warp), (RandomAffineWithInverse, "inverse", inverse)]:
        monkeypatch_like(obj, name, fn)


class _DS(torch.utils.data.Dataset):
    def __getitem__(self, i):
        g = torch.Generator().manual_seed(100 + i)
        return {"img": torch.rand(3, 8, 8, generator=g), "kpts": torch.zeros(2, 2)}

    def __len__(self):
        return 6


def _eval_stages(num_gpus):
    from stablekeypoints_amd import keypoint_regressor as kr, eval as ev
    torch.manual_seed(11)
    idx = kr.find_best_indices(None, None, num_steps=6, device="cpu", top_k=4, furthest_point_num_samples=8,
                               controllers={"cpu": None}, num_gpus=num_gpus, top_k_strategy="gaussian",
                               dataset=_DS())
    img = _DS()[0]["img"]
    tta = ev.run_image_with_context_augmented(None, img, None, torch.tensor([1, 3, 5]), device="cpu",
                                              augmentation_iterations=4, controllers={"cpu": None},
                                              num_gpus=num_gpus, upscale_size=8)
    return idx, tta


def _eval_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        _stub_eval_stages(setattr)
        q.put((rank,) + tuple(t.numpy().copy() for t in _eval_stages(world)))   # by value
    finally:
        dist.destroy_process_group()


def test_two_rank_eval_stages_equal_two_replicas_in_one_process(monkeypatch):
    _stub_eval_stages(monkeypatch.setattr)
    ref_idx, ref_tta = _eval_stages(2)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_eval_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    out = [q.get(timeout=120) for _ in range(2)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, idx, tta in out:
        idx, tta = torch.from_numpy(idx), torch.from_numpy(tta)
        assert torch.equal(idx, ref_idx), (rank, idx, ref_idx)
        assert torch.allclose(tta, ref_tta, rtol=1e-6, atol=1e-7), rank
