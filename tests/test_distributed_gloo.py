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
        q.put((rank, opt.context.detach().clone(), recs))
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
        assert torch.allclose(c, ref_ctx, atol=1e-6, rtol=1e-5), f"rank {rank} context diverged"
        for a, b in zip(recs, ref_recs):
            for k in a:
                assert abs(a[k] - b[k]) <= 1e-5 * max(1.0, abs(b[k])), (k, a[k], b[k])
