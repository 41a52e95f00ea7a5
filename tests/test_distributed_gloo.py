"""Multi-rank semantics of the token optimisation on CPU (gloo, world sizes 2 and 4; 8 for the
sharded step and the eval stages).

The reference runs one replica per GPU under nn.DataParallel and averages the per-replica
losses (optimize.py:428-443).  Here each rank is a process; TokenOptimizer all-reduces the
context gradient (SUM ÷ world) once per optimiser step.  These tests check that sharding the
images over 2 ranks gives the same gradient, loss statistics and Adam update as one rank
processing all of them, using a CPU surrogate for the per-image loss (the real per-image loss
runs on HIP kernels and is covered by tests/test_gpu_parity.py).  SURVEY.md §4 item 5 asks for
2/4/8 ranks; 8 gloo processes do not fit this container's 8 CPUs next to the test runner, so the
CPU suite runs 2 and 4.
"""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


WORLDS = (2, 4)


def _spawn(target, world, *args, timeout=180):
    """Run target(rank, world, port, *args, q) on `world` gloo ranks; return their queue items."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=target, args=(r, world, port) + args + (q,)) for r in range(world)]
    for p in procs:
        p.start()
    out = [q.get(timeout=timeout) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    return out


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


@pytest.mark.parametrize("world", WORLDS + (8,))
def test_sharded_grad_allreduce_equals_single_rank(world):
    n_img, steps = max(4, world), 3
    ref_ctx, ref_recs, _ = _reference_single(n_img, steps)
    out = _spawn(_worker, world, n_img, steps)
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
        return 16   # ≥ 8: every world size below gets whole replica batches


def _eval_stages(num_gpus):
    from stablekeypoints_amd import keypoint_regressor as kr, eval as ev
    torch.manual_seed(11)
    idx = kr.find_best_indices(None, None, num_steps=max(6, num_gpus), device="cpu", top_k=4, furthest_point_num_samples=8,
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


@pytest.mark.parametrize("world", WORLDS + (8,))
def test_sharded_eval_stages_equal_replicas_in_one_process(monkeypatch, world):
    _stub_eval_stages(monkeypatch.setattr)
    ref_idx, ref_tta = _eval_stages(world)
    out = _spawn(_eval_worker, world)
    for rank, idx, tta in out:
        idx, tta = torch.from_numpy(idx), torch.from_numpy(tta)
        assert torch.equal(idx, ref_idx), (rank, idx, ref_idx)
        assert torch.allclose(tta, ref_tta, rtol=1e-6, atol=1e-7), rank


# ---------------------------------------------------------------------------- data order + warps
# optimize.py:356-368 draws each micro-iteration's num_gpus images from ONE shuffled
# DataLoader(batch_size=num_gpus, drop_last=True); replica r gets image r and warp r of that
# batch.  ReplicaSampler / TokenOptimizer.draw_thetas must give rank r exactly those.
def _order_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from stablekeypoints_amd.optimize import ReplicaSampler, TokenOptimizer
        from stablekeypoints_amd.invertable_transform import RandomAffineWithInverse
        torch.manual_seed(1234 + 17 * rank)   # different CPU states: the seed must come from rank 0
        s = ReplicaSampler(7, world, rank)     # seed drawn on rank 0 and broadcast
        picks = [s.next() for _ in range(9)]  # 7 // world groups per epoch (drop_last)
        torch.manual_seed(99 if rank == 0 else 5 + rank)   # ranks seeded differently (bench.py seeds 1234 + rank)
        opt = TokenOptimizer.__new__(TokenOptimizer)
        opt.world, opt.rank = world, rank
        opt.context = torch.zeros(1)
        opt.sync_cpu_rng()                     # as TokenOptimizer.__init__: every rank takes rank 0's CPU stream
        opt.transform = RandomAffineWithInverse(degrees=15, scale=(0.8, 1.0), translate=(0.25, 0.25))
        th = torch.cat([opt.draw_thetas(2), opt.draw_thetas(1)])
        seed = s.gen.initial_seed()
        q.put((rank, picks, th.numpy().copy(), seed))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", WORLDS)
def test_sampler_partitions_each_replica_batch_and_warps_follow_replicas(world):
    from stablekeypoints_amd.optimize import ReplicaSampler
    from stablekeypoints_amd.invertable_transform import RandomAffineWithInverse
    out = sorted(_spawn(_order_worker, world))
    seeds = {o[3] for o in out}
    assert len(seeds) == 1, "ranks shuffled with different seeds"
    # the single-process DataLoader view: one permutation per epoch, groups of `world`, remainder dropped
    gen = torch.Generator().manual_seed(seeds.pop())
    groups = []
    while len(groups) < 9:
        perm = torch.randperm(7, generator=gen).tolist()
        groups += [perm[world * i:world * i + world] for i in range(7 // world)]
    groups = groups[:9]
    for rank, picks, _, _ in out:
        assert picks == [g[rank] for g in groups], (rank, picks, groups)
    for j in range(9):   # each group is split, never duplicated, across the ranks
        assert sorted(o[1][j] for o in out) == sorted(groups[j])
    # warps: the reference draws num_gpus thetas per micro-iteration; replica r uses theta r, from
    # its single CPU generator (rank 0's seed here: the other ranks were seeded differently)
    torch.manual_seed(99)
    ref = RandomAffineWithInverse(degrees=15, scale=(0.8, 1.0), translate=(0.25, 0.25)).draw_theta(3 * world)
    ref = ref.reshape(3, world, 2, 3)
    for rank, _, th, _ in out:
        assert torch.equal(torch.from_numpy(th), ref[:, rank]), rank
    assert ReplicaSampler(5, 1, 0, seed=3).next() == int(torch.randperm(5, generator=torch.Generator().manual_seed(3))[0])


# ---------------------------------------------------------------------------- real step, 2 ranks on one GPU
def _tiny_opt(accum, dev, ctx_shift=0.0):
    """TokenOptimizer on the toy-width SD-1.5 with batching-independent noise (a function of the
    latent), so one image's pass gives the same maps whatever else shares the batch."""
    import recipes
    from stablekeypoints_amd.optimize import TokenOptimizer
    from stablekeypoints_amd.optimize_token import load_ldm
    from stablekeypoints_amd.sd import TINY_CONFIG
    ldm, ctls, _ = load_ldm(dev, "random", feature_upsample_res=32, config=TINY_CONFIG)
    inner = ldm.scheduler

    class Sched:
        timesteps = inner.timesteps

        def add_noise(self, x, noise, t):
            return inner.add_noise(x, torch.sin(7.0 * x), t)
    ldm.scheduler = Sched()
    ctx = torch.from_numpy(recipes.random_logits(52, (1, 16, 32))).to(dev) + ctx_shift
    return TokenOptimizer(ldm, ctls, ctx, top_k=4, furthest_point_num_samples=8, accum=accum, device=dev)


def _tiny_images(dev):
    import recipes
    from stablekeypoints_amd.sd import TINY_IMAGE
    return [torch.from_numpy(recipes.uniform(60 + i, (1, 3, TINY_IMAGE, TINY_IMAGE))).to(dev) for i in range(2)]


def _real_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        dev = "cuda:0"
        torch.cuda.set_device(0)
        torch.manual_seed(5)
        # rank 1 starts from a different embedding: TokenOptimizer must replace it by rank 0's
        opt = _tiny_opt(1, dev, ctx_shift=float(rank))
        img = _tiny_images(dev)[rank]
        idx = opt.micro_steps([img])[0]
        rec = {k: float(v) for k, v in opt.optimizer_step().items()}
        q.put((rank, idx.cpu().numpy().copy(), opt.context.detach().cpu().numpy().copy(), rec))
    finally:
        dist.destroy_process_group()


@pytest.mark.gpu
def test_two_ranks_real_token_opt_step_equals_one_process():
    """TokenOptimizer.micro_steps + optimizer_step on 2 gloo ranks (both on cuda:0, one image
    each) == one process running both images' micro-iterations then Adam (optimize.py:362-448
    with num_gpus=2 vs 1): selected indices exact, loss statistics and the context after Adam
    within 1e-6."""
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    dev = "cuda:0"
    torch.manual_seed(5)
    ref = _tiny_opt(2, dev)
    imgs = _tiny_images(dev)
    ref_idx = [ref.micro_step(imgs[0]), ref.micro_step(imgs[1])]
    ref_rec = {k: float(v) for k, v in ref.optimizer_step().items()}
    ref_ctx = ref.context.detach().cpu()
    del ref
    torch.cuda.empty_cache()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_real_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    out = [q.get(timeout=300) for _ in range(2)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, idx, c, rec in out:
        assert (idx == ref_idx[rank].cpu().numpy()).all(), (rank, idx, ref_idx[rank])
        d = float((torch.from_numpy(c) - ref_ctx).abs().max())
        print(f"\nrank {rank}: context after Adam max|Δ| vs one process {d:.1e}")
        assert d <= 1e-6, d
        for k in rec:
            assert abs(rec[k] - ref_rec[k]) <= 1e-6 * max(1.0, abs(ref_rec[k])), (k, rec[k], ref_rec[k])


# ---------------------------------------------------------------------------- batch_size < world
def _zero_iter_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from stablekeypoints_amd.datasets import SyntheticDataset
        from stablekeypoints_amd.optimize import optimize_embedding
        from stablekeypoints_amd.optimize_token import load_ldm
        from stablekeypoints_amd.sd import TINY_IMAGE
        torch.manual_seed(rank)
        ldm, ctls, num_gpus = load_ldm("cpu", "tiny", feature_upsample_res=16)
        calls = []
        ldm.unet.register_forward_pre_hook(lambda m, i: calls.append(1))
        ctx0 = torch.randn(1, 8, 32, generator=torch.Generator().manual_seed(10 + rank))
        out = optimize_embedding(ldm, context=ctx0.clone(), device="cpu", num_steps=3, batch_size=world - 1,
                                 num_gpus=num_gpus, num_tokens=8, dataset=SyntheticDataset(n=4, size=TINY_IMAGE),
                                 controllers=ctls, top_k=2, furthest_point_num_samples=4, seed=0, log=lambda r: None)
        q.put((rank, num_gpus, len(calls), out.numpy().copy()))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", WORLDS)
def test_batch_size_below_world_runs_zero_iterations(world):
    """optimize.py:362: num_steps·(batch_size // num_gpus) micro-iterations, so batch_size <
    num_gpus optimises nothing.  Every rank returns rank 0's initial
    embedding (broadcast when the optimiser is built) without running the UNet."""
    out = sorted(_spawn(_zero_iter_worker, world))
    ref = torch.randn(1, 8, 32, generator=torch.Generator().manual_seed(10))
    for rank, n, calls, c in out:
        assert n == world and calls == 0, (rank, n, calls)
        assert torch.equal(torch.from_numpy(c), ref), rank
