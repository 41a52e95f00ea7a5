"""Benchmark: StableKeypoints token-optimisation throughput on MI355X (images/sec).

Workload (BASELINE.json configs[1]: "CelebA-wild 512² N=500 tokens, 1×MI355X"): SD-1.5
UNet/VAE with seeded random weights (no checkpoint offline), synthetic 512×512 images
(seeded torch.rand), N=500 tokens × 768, feature_upsample_res=128, the reference's
default hyper-parameters (gaussian top-k 25 → furthest-point 10, σ=2, weights 100/1000,
Adam lr 5e-3, batch_size 4 per GPU).

One "step" = one optimiser step = ``--accum`` (default 4) micro-iterations per rank
(reference optimize.py:362-448), each = 2 captures (image + random affine warp) +
selection + losses + backward through the UNet into the token embedding, then the
gradient all-reduce (RCCL) and Adam.  Weak scaling: every rank processes ``accum``
images per step.  ``value`` = images processed by all ranks ÷ the max-over-ranks time.

Launch: ``python bench.py`` (1 GPU), ``python bench.py --gpus N`` (starts N ranks itself, one per
GPU, RCCL), or ``python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1
bench.py --gpus N`` (the launcher's WORLD_SIZE must equal N).  Rank 0 prints ONE JSON line.
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

HBM_PEAK = 8.0e12          # MI355X_MICROARCH.md: 8.0 TB/s spec
HBM_MEASURED_COPY = 6.29e12
VALU_F32_PEAK = 157.3e12   # MI355X_MICROARCH.md: f32 vector peak (packed v_pk_fma_f32), 256 CUs


class KernelTimer:
    """HIP events around each launch of the named kernels, on the launching (current) stream."""

    def __init__(self, names):
        self.names = set(names)
        self.events = {n: [] for n in names}
        self.nbytes = {n: [] for n in names}
        self.flops = {n: [] for n in names}
        self.cycles = {n: [] for n in names}
        self.enabled = False

    def record(self, name, nbytes, flops=0, cycles=0):
        timer = self

        class _Ctx:
            def __enter__(self_):
                if timer.enabled and name in timer.names:
                    self_.ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
                    self_.ev[0].record()
                else:
                    self_.ev = None
                return self_

            def __exit__(self_, *a):
                if self_.ev is not None:
                    self_.ev[1].record()
                    timer.events[name].append(self_.ev)
                    timer.nbytes[name].append(nbytes)
                    timer.flops[name].append(flops)
                    timer.cycles[name].append(cycles)
                return False
        return _Ctx()

    def summary(self, name):
        ev = self.events[name]
        if not ev:
            return None
        ms = [a.elapsed_time(b) for a, b in ev]
        return {"launches": len(ms), "avg_ms": float(np.mean(ms)), "bytes_per_launch": float(np.mean(self.nbytes[name])),
                "flop_per_launch": float(np.mean(self.flops[name])),
                "issue_cycles_per_launch": float(np.mean(self.cycles[name]))}


# gfx950 VALU issue capacity: 256 CUs × 4 SIMDs at the 2.4 GHz peak engine clock (MI355X_MICROARCH.md)
SIMD_CYCLES_PER_S = 1024 * 2.4e9


def issue_roofline(summary, model):
    """The launch's minimal VALU issue time (its instruction-mix floor: ops.*_issue_cycles over
    1024 SIMDs at 2.4 GHz) against its measured average: the roofline of a kernel whose binding
    resource is VALU ISSUE with 8-cycle transcendentals in the mix, which the packed-FMA FLOP
    peak does not see."""
    cyc = summary.get("issue_cycles_per_launch") or 0.0
    if not cyc:
        return None
    floor_ms = cyc / SIMD_CYCLES_PER_S * 1e3
    return {"floor_ms": floor_ms, "avg_launch_ms": summary["avg_ms"], "frac": floor_ms / summary["avg_ms"],
            "issue_cycles_per_launch": cyc, "model": model}


def _pmc_record(path, name, key, value):
    """(figure, source) for `name` from a profiles/*.json PMC record, only if that record was
    measured on this launch shape (key = (field, expected value)); source names the file, the
    profiled workload and the counter method — the figure is NOT measured in this process."""
    try:
        rec = json.load(open(path)).get(name, {})
    except (OSError, ValueError):
        return None, None
    if rec.get(key[0]) != key[1] or rec.get(value) is None:
        return None, None
    src = {"file": os.path.relpath(path, REPO), "workload": rec.get("workload"), "method": rec.get("method"),
           "measured_in_this_process": False}
    return rec.get(value), src


def _a8_split(dev, T, R, nb=4, reps=20):
    """The A8 call's two launches timed apart (HIP events on the current stream, median of `reps`)
    on synthetic attention-like maps of the bench's shape (a pass's nb images, T tokens, R²), run
    after the timed region: the KL ranking alone (top_k 0) and the ranking of its keys alone."""
    from stablekeypoints_amd import ops
    from stablekeypoints_amd._lib import call, ptr, stream
    g = torch.Generator(device=dev).manual_seed(5)
    maps = torch.rand(nb, T, R, R, device=dev, generator=g) ** 8
    kl = torch.empty(nb, T, device=dev, dtype=torch.float64)
    out = torch.empty(nb, 25, device=dev, dtype=torch.int64)

    def kl_only():
        call("skp_topk_gaussian_batch", ptr(maps), nb, T, R, R, 0, 2.0, 1e-5, 1, ptr(out), ptr(kl), ptr(kl), stream(dev))

    def topk_only():
        call("skp_topk_keys", ptr(kl), nb, T, 25, ptr(out), stream(dev))

    def whole():
        ops.find_top_k_gaussian_batch(maps, 25, sigma=2.0)

    maps_t = torch.rand(nb, T, R, R, device=dev, generator=g) ** 8   # the warps' maps the FPS reads

    def chain_r05():   # KL → rank (skp_topk_gaussian_batch) → argmax + FPS (skp_fps_batch): 4 launches
        c = ops.find_top_k_gaussian_batch(maps, 25, sigma=2.0)
        return ops.furthest_point_sampling_batch(maps_t, 10, c)[0]

    def chain_r06():   # KL → rank + argmax → FPS (ops.gaussian_fps_batch): 3 launches
        return ops.gaussian_fps_batch(maps, maps_t, 25, 10, sigma=2.0)[0]

    if not torch.equal(chain_r05(), chain_r06()):
        raise SystemExit("bench: gaussian_fps_batch differs from the two-call selection")
    res = {}
    for name, fn in (("kl_ms", kl_only), ("topk_ms", topk_only), ("call_ms", whole),
                     ("select_chain_r05_ms", chain_r05), ("select_chain_ms", chain_r06)):
        fn()
        ts = []
        for _ in range(reps):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            fn()
            b.record()
            b.synchronize()
            ts.append(a.elapsed_time(b))
        res[name] = float(np.median(ts))
    res["workload"] = (f"{nb} x ({T}, {R}, {R}) synthetic maps (+ as many warp maps for the FPS), top_k 25, sigma 2, "
                       f"FPS 10; median of {reps}, before the warm-up; select_chain_r05_ms = KL + rank launch + "
                       "argmax + FPS launches (the r05 chain), select_chain_ms = KL + rank/argmax + FPS (r06), "
                       "outputs checked equal")
    del maps, maps_t
    return res


def _sel_bwd_split():
    """Average per-call device time of the sparse backward's phases in the timed region, from the
    HIP events libskp records between its launches on the call's stream (skp_sel_bwd_timing_read),
    or None when no fast-path call was recorded."""
    import ctypes

    from stablekeypoints_amd import _lib
    L = _lib.lib()
    if not hasattr(L, "skp_sel_bwd_timing_read"):
        return None
    ms = (ctypes.c_double * 4)()
    n = ctypes.c_int(0)
    rc = L.skp_sel_bwd_timing_read(ms, ctypes.byref(n))
    L.skp_sel_bwd_timing(0)
    if rc != 0 or n.value == 0:
        return None
    names = ("sel_gather", "sel_doth", "sel_adjv", "sel_dense")
    out = {k: ms[i] / n.value for i, k in enumerate(names)}
    out["calls"] = n.value
    out["timing_source"] = "HIP events recorded by libskp between the phases' launches (skp_sel_bwd_timing)"
    return out


# ------------------------------------------------------------------------------ CPU baseline (port)
def _cgroup_cpus():
    """The job's CPU quota from cgroup v2 ``cpu.max`` ("quota period" or "max period"): raw text and
    quota / period CPUs (None when unlimited or unreadable)."""
    for path in ("/sys/fs/cgroup/cpu.max",):
        try:
            raw = open(path).read().strip()
        except OSError:
            continue
        parts = raw.split()
        cpus = None
        if len(parts) == 2 and parts[0] != "max":
            try:
                cpus = float(parts[0]) / float(parts[1])
            except ValueError:
                cpus = None
        return {"raw": raw, "cpus": cpus}
    return {"raw": None, "cpus": None}


def _cpu_leg_child(threads, tokens, limit_s):
    """bench.py --cpu-leg THREADS in a child process (CPU only: it never initialises HIP), its
    progress on our stderr; returns its JSON result, or {"error": ...} past ``limit_s``."""
    import subprocess
    env = dict(os.environ, OMP_NUM_THREADS=str(threads))
    cmd = [sys.executable, os.path.abspath(__file__), "--cpu-leg", str(threads), "--tokens", str(tokens)]
    try:
        out = subprocess.run(cmd, env=env, stdout=subprocess.PIPE, timeout=limit_s, text=True)
    except subprocess.TimeoutExpired:
        return {"error": f"timed out after {limit_s} s"}
    lines = [l for l in out.stdout.splitlines() if l.startswith("{")]
    return json.loads(lines[-1]) if out.returncode == 0 and lines else {"error": f"rc {out.returncode}"}


def cpu_leg_main(args):
    """--cpu-leg THREADS: one warm-up + one timed micro-iteration of the CPU port at --tokens with
    THREADS torch threads; prints {"value": images/s, "seconds": s}.  Touches no GPU."""
    threads = int(args.cpu_leg)
    torch.set_num_threads(threads)
    rate, dt = cpu_baseline(args, legs_only=True)
    print(json.dumps({"value": rate, "seconds": dt, "threads": threads, "tokens": args.tokens}), flush=True)


def cpu_baseline(args, legs_only=False):
    """One micro-iteration of the same workload on the host CPU: torch-CPU UNet/VAE
    (same architecture and seed) + the numpy oracle for every hot-path row (capture,
    aggregate, selection, losses and their backward).  kind = "port"."""
    from oracle import skp_oracle as O
    from stablekeypoints_amd.sd import build_sd15
    from stablekeypoints_amd.sd.unet import CaptureComplete, attention_core
    from stablekeypoints_amd.datasets import SyntheticDataset

    nproc = os.cpu_count() or 1
    try:
        allowed = len(os.sched_getaffinity(0))   # the CPUs this process may run on
    except AttributeError:
        allowed = nproc
    # OMP_NUM_THREADS, when the host sets it, is the CPU share this job owns (a cgroup quota that
    # neither nproc nor the affinity mask shows); oversubscribing a quota only slows the baseline
    threads = int(os.environ.get("OMP_NUM_THREADS", "0")) or allowed
    if not legs_only:
        torch.set_num_threads(threads)
    ldm = build_sd15(seed=0, device="cpu")
    R = args.res // 4

    class OCapture(torch.autograd.Function):
        @staticmethod
        def forward(ctx, z, s):
            zn = z.detach().numpy()
            a = O.capture_fwd(zn, s, R)
            ctx.zn, ctx.s = zn, s
            return torch.from_numpy(a)

        @staticmethod
        def backward(ctx, g):
            return torch.from_numpy(O.capture_bwd(ctx.zn, ctx.s, R, g.numpy())), None

    class OAggregate(torch.autograd.Function):
        @staticmethod
        def forward(ctx, *layers):
            ctx.shapes = [t.shape for t in layers]
            return torch.from_numpy(O.collect_maps([t.numpy() for t in layers]))

        @staticmethod
        def backward(ctx, g):
            return tuple(torch.from_numpy(np.ascontiguousarray(x))
                         for x in O.collect_maps_bwd(ctx.shapes, g.numpy()))

    class OSharp(torch.autograd.Function):
        @staticmethod
        def forward(ctx, A, sigma):
            l, dA = O.sharpening_loss(A.detach().numpy(), sigma)
            ctx.dA = torch.from_numpy(dA)
            return torch.tensor(l)

        @staticmethod
        def backward(ctx, g):
            return ctx.dA * g, None

    class OEquiv(torch.autograd.Function):
        @staticmethod
        def forward(ctx, A, At, theta):
            l, dA, dAt = O.equivariance_loss(A.detach().numpy(), At.detach().numpy(), theta, 0)
            ctx.g = (torch.from_numpy(dA), torch.from_numpy(dAt))
            return torch.tensor(l)

        @staticmethod
        def backward(ctx, g):
            return ctx.g[0] * g, ctx.g[1] * g, None

    store = []

    def patch(mod):
        def fwd(x, context=None, mask=None):
            B, S, C = x.shape
            q = mod.reshape_heads_to_batch_dim(mod.to_q(x))
            ctxt = x if context is None else context
            k = mod.reshape_heads_to_batch_dim(mod.to_k(ctxt))
            v = mod.reshape_heads_to_batch_dim(mod.to_v(ctxt))
            if context is not None and S <= 1024 and len(store) < 4:
                sim = torch.bmm(q, k.transpose(1, 2)) * mod.scale
                out = torch.bmm(sim.softmax(-1), v)
                store.append(OCapture.apply(sim, int(S ** 0.5)))
            else:
                out = attention_core(q, k, v, mod.scale)
            out = mod.to_out[0](mod.reshape_batch_dim_to_heads(out))
            if len(store) >= 4:
                raise CaptureComplete()
            return out
        return fwd
    for name, child in ldm.unet.named_children():
        if "up" in name:
            for m in child.modules():
                if m.__class__.__name__ == "CrossAttention":
                    m.forward = patch(m)

    torch.manual_seed(0)
    context = torch.randn(1, args.tokens, 768).requires_grad_(True)
    img = SyntheticDataset(n=1, size=args.res, seed=0)[0]["img"][None]

    def capture(image, ctx):
        with torch.no_grad():
            lat = ldm.vae.encode(image * 2 - 1)["latent_dist"].mean * 0.18215
        t = ldm.scheduler.timesteps[-1]
        noisy = ldm.scheduler.add_noise(lat, torch.randn_like(lat), t)
        store.clear()
        try:
            ldm.unet(noisy, t.repeat(1), ctx)
        except CaptureComplete:
            pass
        return OAggregate.apply(*store)

    def micro_iteration(ctx):
        m = capture(img, ctx)
        u = torch.rand(1, 4).numpy()
        theta = O.affine_params(u, 15.0, (0.8, 1.0), (0.25, 0.25))
        timg = torch.from_numpy(O.affine_warp(img.numpy(), theta))
        mt = capture(timg, ctx)
        cand = O.find_top_k_gaussian(m.detach().numpy(), min(25, m.shape[0]), sigma=2.0)
        idx = torch.from_numpy(O.furthest_point_sampling(mt.detach().numpy(), min(10, m.shape[0]), cand))
        sh = OSharp.apply(m[idx], 2.0)
        eq = OEquiv.apply(m[idx], mt[idx], theta)
        loss = (eq * 1000.0 + sh * 100.0) / args.accum
        loss.backward()
        assert ctx.grad is not None and torch.isfinite(ctx.grad).all()

    def timed_rate(ctx, reps):
        micro_iteration(ctx)                         # warm-up (allocator, thread pool, first-touch)
        t0 = time.time()
        for i in range(reps):
            micro_iteration(ctx)
            print(f"cpu_baseline: N={ctx.shape[1]} image {i + 1}/{reps} {time.time() - t0:.1f} s", file=sys.stderr,
                  flush=True)
        return reps / (time.time() - t0), time.time() - t0

    if legs_only:
        return timed_rate(context, 1)
    rate, dt = timed_rate(context, 2)
    # BASELINE.md's small figure: the same micro-iteration at N = 10 tokens (configs[0] scale)
    ctx10 = torch.randn(1, 10, 768).requires_grad_(True)
    rate10, dt10 = timed_rate(ctx10, 2)
    # SURVEY §8(d)'s thread count, os.cpu_count(), as a second figure, in a child process (a fresh
    # OpenMP pool of that size) under a time limit: more threads than the cgroup quota oversubscribe
    # it, and the spinning pool can run many times slower than the quota's thread count
    np_leg = None
    if nproc != threads:
        np_leg = _cpu_leg_child(nproc, 10, limit_s=150)
    cpu = "unknown"
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                cpu = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    quota = _cgroup_cpus()
    return {"value": rate, "unit": "images/sec", "cores": threads, "kind": "port", "nproc": nproc,
            "affinity_cpus": allowed, "cgroup_cpu_max": quota["raw"], "cgroup_cpus": quota["cpus"],
            "threads_source": "OMP_NUM_THREADS" if os.environ.get("OMP_NUM_THREADS") else "sched_getaffinity",
            "value_nproc_threads_N10": np_leg and np_leg.get("value"), "nproc_threads_sample": (
                f"os.cpu_count() = {nproc} threads (child process, OMP_NUM_THREADS={nproc}): "
                + (f"1 image at N=10 after 1 warm-up, {np_leg['seconds']:.1f} s; compare value_N10" if np_leg and
                   np_leg.get("value") else f"did not finish 1 warm-up + 1 image at N=10 within {150} s "
                   f"({np_leg.get('error') if np_leg else 'no result'})")),
            "cpu_model": cpu, "value_N10": rate10,
            "sample": f"2 timed images after 1 warm-up, 1 image = 1 token-opt micro-iteration (2 captures + select + "
                      f"losses + backward), N={args.tokens}, {args.res}²; torch-CPU SD-1.5 UNet/VAE + numpy oracle "
                      f"({threads} threads: OMP_NUM_THREADS if set, else the CPUs this process may use; nproc "
                      f"{nproc}, affinity {allowed}); {dt:.1f} s; "
                      f"value_N10 = the same at N=10 tokens ({dt10:.1f} s)"}


# ------------------------------------------------------------------------------ GPU bench
def _tuned_gemms_in_use():
    from stablekeypoints_amd.tuning import _state
    return bool(_state["loaded"])


# ------------------------------------------------------------------------------ eval-stage benches
FIND_INDICES_T4_ITS = 1.34   # find_best_indices, N=100, upsample 256, 1 image per it, Colab T4


def stage_main(args, ldm, controllers, context, dev, world, rank, backend):
    """--stage find_indices / tta: the no-grad evaluation stages on the fused capture.

    find_indices (keypoint_regressor.find_best_indices, reference keypoint_regressor.py:16-121 with
    main.py:248-267's arguments: upsample_res 256, gaussian top-k 25, σ 2, FPS 10, layers 0-3): one
    step = ``--stage-images`` images per rank, captured in ONE batched VAE/UNet pass, then per image
    top-k + FPS; it/s = images/s (the reference's tqdm "it" is one image at num_gpus = 1).
    tta (keypoint_regressor.precompute_all_keypoints, reference :124-224 with main.py:302-320's
    arguments: 10 augmentations, upscale 512, argmax): one step = ``--stage-images`` images per
    rank, each image's 10 warped copies in one batched pass (with N ranks, each runs 10 // N of every
    image's augmentations, as the reference's replicas do); it/s = images/s.
    Every rank draws the same loader order (one CPU seed) and takes replica ``rank`` of each group,
    as in the reference's DataParallel replicas; value = images of all ranks ÷ max-over-ranks time."""
    from stablekeypoints_amd import keypoint_regressor as kr, ops
    from stablekeypoints_amd.datasets import SyntheticDataset
    n = args.stage_images
    timer = KernelTimer(["skp_capture_maps_fwd", "skp_aggregate", "skp_capture_fwd"])
    ops.set_kernel_timer(timer)
    if args.stage == "find_indices":
        data = SyntheticDataset(n=n * world, size=args.res, seed=7)

        def step():
            return kr.find_best_indices(ldm, context, num_steps=n * world, device=dev, upsample_res=256,
                                        layers=(0, 1, 2, 3), top_k=10, furthest_point_num_samples=25,
                                        controllers=controllers, num_gpus=world, top_k_strategy="gaussian",
                                        sigma=2.0, dataset=data, capture_batch=n)
    else:
        data = SyntheticDataset(n=n, size=args.res, seed=7)
        top = torch.arange(10)

        def step():
            return kr.precompute_all_keypoints(ldm, context, top, device=dev, layers=(0, 1, 2, 3),
                                               augmentation_iterations=10, controllers=controllers,
                                               num_gpus=world, dataset=data, upscale_size=512)

    def barrier():
        if world > 1:
            import torch.distributed as dist
            dist.barrier()
    torch.manual_seed(1234)   # same CPU stream on every rank: loader order and thetas agree
    for _ in range(args.warmup):
        out = step()
    barrier()
    torch.cuda.synchronize()
    timer.enabled = True
    t0 = time.perf_counter()
    for _ in range(args.steps):
        out = step()
    torch.cuda.synchronize()
    barrier()
    elapsed = time.perf_counter() - t0
    timer.enabled = False
    if world > 1:
        import torch.distributed as dist
        t = torch.tensor([elapsed], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    # find_indices shards the images over the ranks (weak); tta splits each image's augmentations
    # over the ranks (the reference's augmentation_iterations // num_gpus per replica: strong)
    images = (world * n if args.stage == "find_indices" else n) * args.steps
    value = images / elapsed
    roof = None
    fw = timer.summary("skp_capture_maps_fwd")
    if fw:
        t = fw["avg_ms"] * 1e-3
        flops = fw["flop_per_launch"]
        roof = {"kernel": "skp_capture_maps_fwd", "bound": "valu", "achieved": flops / t / 1e12,
                "peak": VALU_F32_PEAK / 1e12, "unit": "TFLOP/s", "frac": flops / t / VALU_F32_PEAK, "traffic": None,
                "avg_launch_ms": fw["avg_ms"], "launches": fw["launches"],
                "timing_source": "HIP events around every launch in the timed region (bench.py KernelTimer)",
                "algorithmic_flop_per_launch": flops, "algorithmic_bytes_per_launch": fw["bytes_per_launch"],
                "hbm_achieved_GBps": fw["bytes_per_launch"] / t / 1e9,
                "flop_model": "15 FLOP per (image, head, layer, pixel, token) + 8 per (row, low-res column, token); "
                              "ops.capture_maps_flops",
                "issue_roofline": issue_roofline(fw, "ops.capture_maps_issue_cycles")}
    if rank == 0:
        if args.stage == "find_indices":
            metric = f"it/s (find_best_indices, {args.res}², N={args.tokens} tokens, 1 image per it)"
            workload = (f"keypoint_regressor.find_best_indices: SD-1.5 fp32, {args.res}², N={args.tokens}, "
                        f"feature_upsample_res={args.upsample_res}, upsample_res 256, gaussian top-25 (σ 2) -> FPS 10, "
                        f"{n} images per rank per batched capture pass")
            vs = value / FIND_INDICES_T4_ITS if args.tokens == 100 and args.res == 512 else None
        else:
            metric = f"it/s (precompute_all_keypoints, {args.res}², 10 augmentations, 1 image per it)"
            workload = (f"keypoint_regressor.precompute_all_keypoints: SD-1.5 fp32, {args.res}², N={args.tokens}, "
                        f"feature_upsample_res={args.upsample_res}, 10 tokens, 10 augmentations per image in one "
                        "batched capture pass, upscale 512, argmax")
            vs = None
        line = {"metric": metric, "value": value, "unit": "it/s", "n_gpus": world, "steps": args.steps,
                "warmup": args.warmup, "ms_per_step": elapsed / args.steps * 1e3, "higher_is_better": True,
                "scaling": "weak" if args.stage == "find_indices" else "strong", "vs_baseline": vs,
                "vs_baseline_source": ("BASELINE.md: 1.34 it/s, Colab T4, StableKeypoints.ipynb:2724" if vs else None),
                "dtype": "f32", "data": f"synthetic (seeded torch.rand {args.res}² images, random-init SD15)",
                "config": {"workload": workload, "stage": args.stage, "images_per_step": images // args.steps,
                           "tokens": args.tokens, "image_res": args.res,
                           "parallelism": (f"dp{world} (replicas; {'RCCL' if backend == 'nccl' else backend} "
                                           "all_gather / all-reduce at the end)" if world > 1 else "dp1"),
                           "tuned_gemms": _tuned_gemms_in_use()},
                "roofline": roof, "cpu_baseline": None}
        print(json.dumps(line), flush=True)
    if world > 1:
        import torch.distributed as dist
        dist.destroy_process_group()


def dry_run_main(world, rank, local):
    """--dry-run: the launch path without the GPU.  Every rank joins a gloo group (when world > 1),
    the ranks all-gather what they saw, and rank 0 prints one JSON line."""
    seen = {"rank": rank, "world_env": world, "local_rank": local, "device": f"cuda:{local}", "pid": os.getpid()}
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("gloo")
        ranks = [None] * dist.get_world_size()
        dist.all_gather_object(ranks, seen)
        n = dist.get_world_size()
        dist.destroy_process_group()
    else:
        ranks, n = [seen], 1
    if rank == 0:
        print(json.dumps({"dry_run": True, "n_gpus": n, "ranks": ranks}), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--model", default="sd15", choices=["sd15", "sdxl"],
                    help="sdxl = BASELINE.json configs[4] (SDXL UNet, 1024², context width 2048; not the headline)")
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--accum", type=int, default=4, help="images per rank per optimiser step (batch_size/num_gpus)")
    ap.add_argument("--tokens", type=int, default=500)
    ap.add_argument("--res", type=int, default=512)
    ap.add_argument("--upsample-res", type=int, default=128)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--conv-benchmark", type=int, default=0, help="torch.backends.cudnn.benchmark (MIOpen exhaustive find)")
    ap.add_argument("--conv", default="wino", choices=["wino", "miopen"],
                    help="3x3 stride-1 convolutions: skp_conv3x3_wino where eligible, or MIOpen throughout")
    ap.add_argument("--attn-backend", default="math", choices=["math", "sdpa"],
                    help="un-captured UNet attention: explicit fp32 GEMM+softmax (math) or torch SDPA")
    ap.add_argument("--micro-batch", type=int, default=0,
                    help="images per VAE/UNet pass (0 = all `accum` images of an optimiser step in one pass)")
    ap.add_argument("--prefetch", type=int, default=0,
                    help="VAE-encode the next PREFETCH passes' images on a side stream (TokenOptimizer.prefetch), "
                         "enqueued between the current pass's forward and backward; steady state: every timed step "
                         "runs one UNet pass and one VAE pass, the warm-up's prefetches are balanced by the last "
                         "timed steps' (0 = no prefetch: each pass encodes its own images on the main stream, "
                         "measured 0.3-0.5%% faster than 1 on the current tree in three A/B sessions, "
                         "profiles/r03ar_prefetch_ab.txt, profiles/r03at_ab.txt: the GPU is saturated either way "
                         "and the side stream's large convolutions delay the UNet's small launches)")
    ap.add_argument("--prefetch-at", default="capture_bwd", choices=["capture_bwd", "bwd"],
                    help="where the VAE prefetch is enqueued: after the sparse capture backward (the VAE overlaps "
                         "the UNet backward) or before the whole backward")
    ap.add_argument("--graph", type=int, default=0,
                    help="1 = replay each pass (capture forward, selection, losses, backward into the embedding) as "
                         "one captured HIP graph (TokenOptimizer(graph=True)); measured neutral at the bench shape "
                         "(39.47 vs 39.50 images/s, profiles/r03t_graph_ab.txt: the GPU, not the host, is the bound), "
                         "so eager launches stay the default")
    ap.add_argument("--gc-freeze", type=int, default=1, help="gc.freeze() after the model is built (host overhead)")
    ap.add_argument("--stage", default="token_opt", choices=["token_opt", "find_indices", "tta"],
                    help="token_opt = the headline token-optimisation step; find_indices = "
                         "keypoint_regressor.find_best_indices (no-grad capture at upsample 256, gaussian top-25 -> "
                         "FPS 10), one step = --stage-images images per rank in one batched pass; tta = "
                         "precompute_all_keypoints (10 augmentations at 512, argmax), one step = --stage-images images")
    ap.add_argument("--stage-images", type=int, default=8, help="images per rank per step of a --stage bench")
    ap.add_argument("--traffic", default=os.path.join(REPO, "profiles", "pmc_traffic.json"),
                    help="JSON with PMC-derived HBM bytes per launch of the roofline kernel")
    ap.add_argument("--cpu-leg", type=int, default=0, help=argparse.SUPPRESS)
    ap.add_argument("--dry-run", action="store_true",
                    help="launch path only: start the --gpus ranks, join them over gloo, print one JSON line with the "
                         "world each rank saw and the device it would use; no HIP call anywhere")
    args = ap.parse_args()
    if args.cpu_leg:
        return cpu_leg_main(args)
    if args.graph and args.prefetch < 1:
        args.prefetch = 1   # only prefetched passes replay a graph (TokenOptimizer.micro_steps)

    # --gpus N means N ranks.  Without a launcher environment and N > 1, this process starts them
    # (torch.distributed.run as a child, before any HIP call) and exits with their status; under a
    # launcher, its world must be the N asked for.
    from stablekeypoints_amd.launch import launcher_env, spawn_ranks
    env = launcher_env()
    if env is None and args.gpus > 1:
        sys.exit(spawn_ranks(args.gpus, [os.path.abspath(__file__)], sys.argv[1:]))
    world, rank, local = env if env is not None else (1, 0, 0)
    if world != args.gpus:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but the launcher started WORLD_SIZE={world} ranks")
    # Rehearsal of the multi-GPU path on a one-GPU box (not the measured configuration):
    # SKP_BENCH_ONE_DEVICE=1 puts every rank on cuda:0, SKP_BENCH_DIST_BACKEND=gloo replaces RCCL
    # (which refuses two ranks on one device).  The driver's N-GPU runs use neither.
    if os.environ.get("SKP_BENCH_ONE_DEVICE") == "1":
        local = 0
    backend = os.environ.get("SKP_BENCH_DIST_BACKEND", "nccl")
    if args.dry_run:
        return dry_run_main(world, rank, local)
    if world > 1:
        import torch.distributed as dist
        torch.cuda.set_device(local)
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
        world = dist.get_world_size()
        backend = dist.get_backend()
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)

    from stablekeypoints_amd import ops
    from stablekeypoints_amd.sd.unet import CrossAttention
    from stablekeypoints_amd.optimize import TokenOptimizer
    CrossAttention.backend = args.attn_backend
    torch.backends.cudnn.benchmark = bool(args.conv_benchmark)
    if args.conv == "miopen":
        ops.WINO_MIN_WORKGROUPS = 1 << 30
    from stablekeypoints_amd.optimize_token import load_ldm
    from stablekeypoints_amd.datasets import SyntheticDataset

    if args.model == "sdxl" and args.res == 512:
        args.res = 1024
    # explicit seeded random weights (load_ldm raises for a hub name it cannot load offline)
    ldm, controllers, num_gpus = load_ldm(dev, "random-xl" if args.model == "sdxl" else "random",
                                          feature_upsample_res=args.upsample_res)
    if args.gc_freeze:
        import gc
        gc.collect()
        gc.freeze()   # the model's ~10^5 long-lived objects leave the cyclic collector's scans
    torch.manual_seed(0)
    context = torch.randn(1, args.tokens, ldm.unet.cross_attention_dim).to(dev)
    if args.stage != "token_opt":
        return stage_main(args, ldm, controllers, context.detach(), dev, world, rank, backend)
    torch.manual_seed(1234 + rank)
    opt = TokenOptimizer(ldm, controllers, context, accum=args.accum, device=dev, graph=bool(args.graph))
    opt.prefetch_at = args.prefetch_at
    data = SyntheticDataset(n=16, size=args.res, seed=rank)
    imgs = [data[i]["img"][None].to(dev) for i in range(len(data))]
    timer = KernelTimer(["skp_aggregate", "skp_capture_fwd", "skp_capture_bwd", "skp_capture_maps_fwd",
                         "skp_capture_maps_bwd", "skp_capture_maps_bwd_sel", "skp_topk_gaussian_batch",
                         "skp_topk_keys", "skp_selection"])
    ops.set_kernel_timer(timer)

    counter = [0]

    mb = args.micro_batch if args.micro_batch > 0 else args.accum

    def batch_at(c, n):
        return [imgs[(c + i) % len(imgs)] for i in range(n)]

    def step():
        done = 0
        while done < args.accum:
            n = min(mb, args.accum - done)
            cur = batch_at(counter[0], n)
            ahead = []
            if args.prefetch:
                opt.prefetch(cur)                                   # no-op when already prefetched
                ahead = [batch_at(counter[0] + d * n, min(mb, args.accum)) for d in range(1, args.prefetch + 1)]
            # the next passes' VAE is enqueued between this pass's forward and backward
            opt.micro_steps(cur, prefetch=ahead)
            counter[0] += n
            done += n
        return opt.optimizer_step()

    def barrier():
        if world > 1:
            import torch.distributed as dist
            dist.barrier()

    # the A8 call's launches timed apart in isolation, before the warm-up (kept out of the traces'
    # timed region)
    a8_split = _a8_split(dev, args.tokens, args.upsample_res) if args.model == "sd15" else None
    for _ in range(args.warmup):
        step()
    barrier()
    torch.cuda.synchronize()
    timer.enabled = True
    from stablekeypoints_amd import _lib
    if hasattr(_lib.lib(), "skp_sel_bwd_timing"):
        _lib.lib().skp_sel_bwd_timing(1)   # per-phase events inside the sparse backward (split below)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        rec = step()
    torch.cuda.synchronize()
    barrier()
    elapsed = time.perf_counter() - t0
    timer.enabled = False
    sel_split = _sel_bwd_split()
    if world > 1:
        import torch.distributed as dist
        t = torch.tensor([elapsed], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    images = world * args.accum * args.steps
    value = images / elapsed
    timing_src = ("HIP events around every launch in the timed region, on the launching stream "
                  "(bench.py KernelTimer); launches that overlap the side-stream VAE prefetch share the GPU "
                  "with it (isolated launch times: tools/kbench.py)")
    if args.graph:
        # the timed steps replay a HIP graph, which runs no Python and so records no per-kernel
        # events: the same pass runs once eagerly after the timed region (same shapes, same
        # kernels) with the events around every libskp launch
        opt.graph = False
        timer.enabled = True
        step()
        torch.cuda.synchronize()
        timer.enabled = False
        timing_src = ("HIP events around every launch of one eager pass run after the timed region (the timed "
                      "steps replay a HIP graph of the same kernels), on the launching stream (bench.py KernelTimer)")

    # roofline: the dominant hot-path kernel, skp_capture_maps_fwd (fused capture + per-image
    # aggregate), is VALU-bound (bicubic taps + exp + normalise per (pixel, token, layer, head));
    # its HBM traffic is reported beside it.  With ops.FUSED_MAPS = False the r01 path's HBM-bound
    # skp_aggregate is reported instead.
    roof = None
    extra = {}
    fw = timer.summary("skp_capture_maps_fwd")
    valu_json = os.path.join(REPO, "profiles", "pmc_valu.json")
    if fw:
        flops = fw["flop_per_launch"]   # ops.capture_maps_flops of the launch's (B, H, N, R, sizes)
        t = fw["avg_ms"] * 1e-3
        traffic, traffic_src = _pmc_record(args.traffic, "skp_capture_maps_fwd",
                                           ("algorithmic_bytes_per_launch", fw["bytes_per_launch"]),
                                           "hbm_bytes_per_launch")
        vb, vb_src = _pmc_record(valu_json, "skp_capture_maps_fwd", ("flop_per_launch", flops), "valu_busy")
        roof = {"kernel": "skp_capture_maps_fwd", "bound": "valu", "achieved": flops / t / 1e12,
                "peak": VALU_F32_PEAK / 1e12, "unit": "TFLOP/s", "frac": flops / t / VALU_F32_PEAK,
                "traffic": traffic, "traffic_source": traffic_src, "avg_launch_ms": fw["avg_ms"],
                "launches": fw["launches"], "timing_source": timing_src,
                "algorithmic_flop_per_launch": flops, "algorithmic_bytes_per_launch": fw["bytes_per_launch"],
                "hbm_achieved_GBps": fw["bytes_per_launch"] / t / 1e9,
                "hbm_frac": fw["bytes_per_launch"] / t / HBM_PEAK,
                "valu_busy_pmc": vb, "valu_busy_source": vb_src,
                "flop_model": "15 FLOP per (image, head, layer, pixel, token) + 8 per (row, low-res column, token); "
                              "ops.capture_maps_flops",
                "issue_roofline": issue_roofline(fw, "ops.capture_maps_issue_cycles: per (image, head, layer, pixel, "
                                                     "token) 4 packed tap FMAs, ½ v_max3, 1 packed FMA, 1 v_exp_f32 "
                                                     "(8 cycles), 1 packed add, 1 packed FMA")}
    for name, model in (("skp_capture_maps_bwd_sel", "20 FLOP per (image, head, layer, pixel, token) + 16 per (row, "
                         "low-res column, token): the dense part; ops.capture_maps_sel_bwd_flops"),
                        ("skp_capture_maps_bwd", "24 FLOP per (image, head, layer, pixel, token) + 16 per (row, "
                         "low-res column, token); ops.capture_maps_bwd_flops")):
        bw = timer.summary(name)
        if bw:
            t = bw["avg_ms"] * 1e-3
            vb, vb_src = _pmc_record(valu_json, name, ("flop_per_launch", bw["flop_per_launch"]), "valu_busy")
            extra[name] = {"bound": "valu", "avg_ms": bw["avg_ms"], "launches": bw["launches"],
                           "timing_source": timing_src, "achieved": bw["flop_per_launch"] / t / 1e12,
                           "peak": VALU_F32_PEAK / 1e12, "unit": "TFLOP/s",
                           "frac": bw["flop_per_launch"] / t / VALU_F32_PEAK,
                           "algorithmic_flop_per_call": bw["flop_per_launch"], "flop_model": model,
                           "GB/s_algorithmic": bw["bytes_per_launch"] / t / 1e9,
                           "algorithmic_bytes_per_call": bw["bytes_per_launch"],
                           "valu_busy_pmc": vb, "valu_busy_source": vb_src,
                           "issue_roofline": issue_roofline(bw, "ops.capture_maps_sel_bwd_issue_cycles (the dense part)")}
            if name == "skp_capture_maps_bwd_sel" and sel_split:
                extra[name]["split_ms"] = sel_split
    agg = timer.summary("skp_aggregate")
    if agg:
        achieved = agg["bytes_per_launch"] / (agg["avg_ms"] * 1e-3)
        traffic, traffic_src = _pmc_record(args.traffic, "skp_aggregate",
                                           ("algorithmic_bytes_per_launch", agg["bytes_per_launch"]),
                                           "hbm_bytes_per_launch")
        rec_a = {"kernel": "skp_aggregate", "bound": "hbm", "achieved": achieved / 1e9, "peak": HBM_PEAK / 1e9,
                 "unit": "GB/s", "frac": achieved / HBM_PEAK, "traffic": traffic, "traffic_source": traffic_src,
                 "avg_launch_ms": agg["avg_ms"], "launches": agg["launches"],
                 "algorithmic_bytes_per_launch": agg["bytes_per_launch"],
                 "frac_of_measured_copy": achieved / HBM_MEASURED_COPY}
        if roof is None:
            roof = rec_a
        else:
            extra["skp_aggregate"] = rec_a
    sel = timer.summary("skp_topk_gaussian_batch")
    if sel:
        achieved = sel["bytes_per_launch"] / (sel["avg_ms"] * 1e-3)
        traffic, traffic_src = _pmc_record(args.traffic, "skp_topk_gaussian_batch",
                                           ("algorithmic_bytes_per_launch", sel["bytes_per_launch"]),
                                           "hbm_bytes_per_launch")
        extra["skp_topk_gaussian_batch"] = {
            "bound": "hbm", "avg_ms": sel["avg_ms"], "launches": sel["launches"], "timing_source": timing_src,
            "achieved": achieved / 1e9, "peak": HBM_PEAK / 1e9, "unit": "GB/s", "frac": achieved / HBM_PEAK,
            "algorithmic_bytes_per_launch": sel["bytes_per_launch"], "traffic": traffic, "traffic_source": traffic_src,
            "note": "the KL keys of a pass's images (kl_gauss_stream_kernel), one launch; r06: the ranking of the "
                    "keys moved into the candidates' argmax launch (skp_fps_keys_batch), timed in `selection`"}
        extra["a8_call_ms"] = sel["avg_ms"]
        extra["a8_split_isolated"] = a8_split
    chain = timer.summary("skp_selection")
    if chain:
        extra["selection"] = {"avg_ms": chain["avg_ms"], "launches": chain["launches"], "timing_source": timing_src,
                              "note": "a pass's whole selection, one timed scope: KL keys → ranking + the 25 candidates' "
                                      "argmax on the warps' maps → FPS (3 launches; r05: 4)"}
    for k in ("skp_capture_fwd", "skp_capture_bwd"):
        s_ = timer.summary(k)
        if s_:
            extra[k] = {"avg_ms": s_["avg_ms"], "launches": s_["launches"],
                        "GB/s_algorithmic": s_["bytes_per_launch"] / (s_["avg_ms"] * 1e-3) / 1e9}

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline and args.model == "sd15":
        ops.set_kernel_timer(None)
        cpu = cpu_baseline(args)

    if rank == 0:
        if args.model == "sdxl":
            metric = f"images/sec (token-opt step, {args.res}², N={args.tokens} tokens, SDXL)"
            workload = (f"SDXL-shaped {args.res}², N={args.tokens} tokens, SDXL UNet fp32 (20 heads x 64 at the 32² "
                        f"capture layers, context width 2048), feature_upsample_res={args.upsample_res} "
                        "(BASELINE.json configs[4])")
        else:
            metric = "images/sec (token-opt step, 512², N=500 tokens)"
            workload = ("CelebA-wild-shaped 512², N=500 tokens, SD-1.5 fp32, feature_upsample_res=128, "
                        "batch_size 4 per GPU (BASELINE.json configs[1]); the 4 images and their warps "
                        "in one VAE/UNet pass of 8")
        out = {"metric": metric, "value": value, "unit": "images/sec",
               "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
               "ms_per_step": elapsed / args.steps * 1e3, "higher_is_better": True, "scaling": "weak",
               "vs_baseline": None, "dtype": "f32",
               "data": f"synthetic (seeded torch.rand {args.res}² images, random-init {args.model.upper()})",
               "config": {"workload": workload,
                          "global_batch": world * args.accum, "tokens": args.tokens, "image_res": args.res,
                          "feature_upsample_res": args.upsample_res, "micro_batch": mb,
                          "parallelism": (f"dp{world} ({'RCCL' if backend == 'nccl' else backend} all-reduce of the "
                                          "token-embedding gradient)" if world > 1 else "dp1 (single process, no collective)"),
                          "tuned_gemms": _tuned_gemms_in_use(), "hip_graph": opt._g is not None,
                          "vae_prefetch": args.prefetch, "prefetch_at": args.prefetch_at},
               "roofline": roof, "cpu_baseline": cpu, "kernels": extra,
               "last_loss": float(rec["loss"])}
        print(json.dumps(out), flush=True)
    if world > 1:
        import torch.distributed as dist
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
