"""Generate golden vectors by importing the REFERENCE implementation (build container only).

Run:  PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_goldens.py

The reference (damaggu/StableKeypoints, read-only at /root/reference) is imported at
function level with stubs for packages absent here (wandb, h5py, cv2, diffusers,
torchvision) and a namespace package for its ``datasets/`` folder.
Its hot-path functions run on torch-CPU; their outputs are written as small
``.npz`` fixtures next to this script.  Large inputs are regenerated from the
numpy recipes in ``recipes.py`` and pinned by SHA-256.  The reference itself never
leaves this container: nothing under ``tests/`` imports it at test time.

This script refuses to run when /root/reference is absent (e.g. on the GPU box).
"""
import os
import sys
import types
from unittest.mock import MagicMock

import numpy as np

REF = "/root/reference"
HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))


def import_reference():
    if not os.path.isdir(os.path.join(REF, "unsupervised_keypoints")):
        raise SystemExit("make_goldens: /root/reference is absent; goldens are generated only in the build container")
    sys.dont_write_bytecode = True
    for m in ["wandb", "h5py", "cv2", "diffusers", "torchvision", "torchvision.transforms",
              "torchvision.transforms.functional", "torchvision.datasets"]:
        sys.modules[m] = MagicMock()
    ds = types.ModuleType("datasets")
    ds.__path__ = [os.path.join(REF, "datasets")]
    sys.modules["datasets"] = ds
    # The reference's package has no __init__.py: this repo's own `unsupervised_keypoints` alias
    # (a regular package) would shadow the namespace package, so pin the reference's path.
    uk = types.ModuleType("unsupervised_keypoints")
    uk.__path__ = [os.path.join(REF, "unsupervised_keypoints")]
    sys.modules["unsupervised_keypoints"] = uk
    sys.path.insert(0, REF)
    from unsupervised_keypoints import ptp_utils, optimize, eval as ref_eval, optimize_token, invertable_transform
    from unsupervised_keypoints import keypoint_regressor
    for m in (ptp_utils, optimize, ref_eval, invertable_transform, keypoint_regressor):
        assert os.path.abspath(m.__file__).startswith(REF), m.__file__
    return types.SimpleNamespace(ptp_utils=ptp_utils, optimize=optimize, eval=ref_eval,
                                 optimize_token=optimize_token, invertable_transform=invertable_transform,
                                 keypoint_regressor=keypoint_regressor)


sys.path.insert(0, HERE)
sys.path.insert(0, REPO)
import recipes  # noqa: E402
import torch  # noqa: E402
import torch.nn as nn  # noqa: E402

LAYER_SHAPES_SMALL = [(4, 64), (4, 64), (4, 64), (8, 32)]      # (s, C) per captured layer
LAYER_SHAPES_SD15 = [(16, 1280), (16, 1280), (16, 1280), (32, 640)]
HEADS = 8


def _np(t):
    return t.detach().cpu().numpy()


class _UpTree(nn.Module):
    """Module tree with an ``up_blocks`` child holding CrossAttention modules.

    The reference's ``register_attention_control`` only walks children whose name
    contains "up" (ptp_utils.py:564-568) and patches class name "CrossAttention".
    """

    def __init__(self, shapes, ctx_dim, params):
        super().__init__()
        from stablekeypoints_amd.sd.unet import CrossAttention
        self.up_blocks = nn.ModuleList()
        for li, (s, c) in enumerate(shapes):
            m = CrossAttention(c, cross_attention_dim=ctx_dim, heads=HEADS, dim_head=c // HEADS)
            m.load_state_dict({k: torch.from_numpy(v) for k, v in params[li].items()})
            self.up_blocks.append(m)


def capture_case(R, shapes, n_tokens, ctx_dim, seed, want_grad, indices=None, upsample_res=-1, layers=(0, 1, 2, 3)):
    ref = REFM
    xs_np, ctx_np, params = recipes.capture_inputs(seed, shapes, n_tokens, ctx_dim)
    tree = _UpTree(shapes, ctx_dim, params)
    ctl = ref.ptp_utils.AttentionStore()
    ref.ptp_utils.register_attention_control(tree, ctl, feature_upsample_res=R)
    xs = [torch.from_numpy(x).requires_grad_(want_grad) for x in xs_np]
    ctx = torch.from_numpy(ctx_np).requires_grad_(want_grad)
    outs = [m(x, context=ctx) for m, x in zip(tree.up_blocks, xs)]
    attn = [a for a in ctl.step_store["attn"]]
    maps = ref.optimize.collect_maps(ctl, from_where=["up_cross"], upsample_res=upsample_res, layers=list(layers),
                                     indices=indices)
    return tree, xs, ctx, outs, attn, maps


def gen_capture_small():
    out = {}
    R, N, D = 32, 16, 24
    tree, xs, ctx, outs, attn, maps = capture_case(R, LAYER_SHAPES_SMALL, N, D, seed=1, want_grad=True)
    wsel = torch.zeros_like(maps)
    sel = [3, 7, 11]
    wsel[sel] = torch.from_numpy(recipes.random_logits(5, (len(sel), R, R)))
    loss = (maps * wsel).sum() + sum((o ** 2).mean() for o in outs) * 0.0
    loss.backward()
    out["R"] = R
    out["N"] = N
    out["ctx"] = _np(ctx)
    for i, x in enumerate(xs):
        out[f"x{i}"] = _np(x)
        out[f"dx{i}"] = _np(x.grad)
        out[f"attn{i}"] = _np(attn[i])
        out[f"out{i}"] = _np(outs[i])
        for name, p in tree.up_blocks[i].named_parameters():
            out[f"w{i}.{name}"] = _np(p)
    out["dctx"] = _np(ctx.grad)
    out["map"] = _np(maps)
    out["wsel"] = _np(wsel)
    # index gather + bilinear up-res + layer subset (collect_maps optimize.py:44-75)
    *_, maps_b = capture_case(R, LAYER_SHAPES_SMALL, N, D, seed=1, want_grad=False,
                              indices=[5, 0, 9], upsample_res=48, layers=[0, 2, 3])
    out["map_idx_up48_l023"] = _np(maps_b)
    np.savez_compressed(os.path.join(HERE, "capture_small.npz"), **out)


def gen_capture_sd15():
    """Full-shape capture+aggregate (N=500, R=128): argmax, per-token sums, samples only."""
    R, N, D = 128, 500, 768
    with torch.no_grad():
        *_, maps = capture_case(R, LAYER_SHAPES_SD15, N, D, seed=3, want_grad=False)
    m = _np(maps)
    out = {"R": R, "N": N,
           "argmax_rc": _np(REFM.eval.find_max_pixel(maps)),
           "token_sums": m.reshape(N, -1).sum(axis=1, dtype=np.float64),
           "samples_idx": np.arange(0, m.size, 9973, dtype=np.int64)}
    out["samples"] = m.reshape(-1)[out["samples_idx"]]
    top2 = np.sort(m.reshape(N, -1), axis=1)[:, -2:]
    out["argmax_margin"] = (top2[:, 1] - top2[:, 0]).astype(np.float32)
    np.savez_compressed(os.path.join(HERE, "capture_sd15.npz"), **out)


def gen_argmax():
    ev = REFM.eval
    out = {}
    cases = torch.from_numpy(recipes.argmax_edge_cases())
    out["edge"] = _np(cases)
    out["edge_max"] = _np(ev.find_max_pixel(cases.clone()))
    out["edge_k3"] = _np(ev.find_k_max_pixels(cases.clone(), num=3))
    m = torch.from_numpy(recipes.attention_like_maps(11, 6, 32))
    out["maps32"] = _np(m)
    out["maps32_k3"] = _np(ev.find_k_max_pixels(m.clone(), num=3))
    pt = ev.find_max_pixel(m)
    out["maps32_mask"] = _np(ev.mask_radius(m.clone(), pt, 0.05 * 32 * 3))
    wa = m.clone()
    out["maps32_wavg"] = _np(ev.pixel_from_weighted_avg(wa, distance=5))
    out["maps32_wavg_mutated"] = _np(wa)
    out["maps32_wavg_nodist"] = _np(ev.pixel_from_weighted_avg(m.clone(), distance=-1))
    big = torch.from_numpy(recipes.attention_like_maps(12, 10, 512))
    out["maps512_sha"] = np.array(recipes.sha256(_np(big)))
    out["maps512_max"] = _np(ev.find_max_pixel(big))
    out["maps512_wavg"] = _np(ev.pixel_from_weighted_avg(big.clone()))
    np.savez_compressed(os.path.join(HERE, "argmax.npz"), **out)


def gen_gaussian():
    ot = REFM.optimize_token
    out = {}
    pos = torch.from_numpy(recipes.uniform(21, (2, 5, 2)))
    out["pos"] = _np(pos)
    for size, sigma in ((32, 2.0), (128, 2.0), (20, 3.0)):
        out[f"circles_{size}_{sigma}"] = _np(ot.gaussian_circles(pos, size=size, sigma=sigma, device="cpu"))
    out["circle_32_2.0"] = _np(ot.gaussian_circle(pos[0], size=32, sigma=2.0, device="cpu"))
    np.savez_compressed(os.path.join(HERE, "gaussian.npz"), **out)


def gen_select():
    pu = REFM.ptp_utils
    out = {}
    # full-shape selection (A8/A9/A10) from regenerated maps
    maps = torch.from_numpy(recipes.attention_like_maps(31, 500, 128))
    maps_t = torch.from_numpy(recipes.attention_like_maps(32, 500, 128))
    out["maps_sha"] = np.array(recipes.sha256(_np(maps)))
    out["maps_t_sha"] = np.array(recipes.sha256(_np(maps_t)))
    cand = pu.find_top_k_gaussian(maps, 25, sigma=2.0)
    out["topk_gauss25"] = _np(cand)
    out["topk_gauss25_s2"] = _np(pu.find_top_k_gaussian(maps, 25, sigma=2.0, num_subjects=2))
    out["entropy25"] = _np(pu.entropy_sort(maps, 25))
    out["entropy25_sharp"] = _np(pu.entropy_sort(maps * 100.0, 25))
    out["fps10"] = _np(pu.furthest_point_sampling(maps_t, 10, cand))
    out["fps10_same"] = _np(pu.furthest_point_sampling(maps, 10, cand))
    # small committed case
    ms = torch.from_numpy(recipes.attention_like_maps(33, 64, 32))
    out["maps_small"] = _np(ms)
    c = pu.find_top_k_gaussian(ms, 12, sigma=2.0)
    out["small_topk12"] = _np(c)
    out["small_entropy12"] = _np(pu.entropy_sort(ms, 12))
    out["small_fps5"] = _np(pu.furthest_point_sampling(ms, 5, c))
    # FPS with tied positions: all candidates share one argmax
    tie = torch.zeros(6, 8, 8)
    tie[:, 3, 4] = 1.0
    tie[4, 0, 0] = 2.0
    out["tie_maps"] = _np(tie)
    out["tie_fps4"] = _np(pu.furthest_point_sampling(tie, 4, torch.tensor([5, 2, 4, 0, 1])))
    np.savez_compressed(os.path.join(HERE, "select.npz"), **out)


def gen_losses():
    opt = REFM.optimize
    it = REFM.invertable_transform
    out = {}
    A = torch.from_numpy(recipes.attention_like_maps(41, 10, 32)).requires_grad_(True)
    At = torch.from_numpy(recipes.attention_like_maps(42, 10, 32)).requires_grad_(True)
    out["A"] = _np(A)
    out["At"] = _np(At)
    for ns in (1, 2):
        A.grad = None
        l = opt.sharpening_loss(A, sigma=2.0, device="cpu", num_subjects=ns)
        l.backward()
        out[f"sharp_ns{ns}"] = _np(l)
        out[f"dA_sharp_ns{ns}"] = _np(A.grad)
    # equivariance (optimize.py:157-163) with two replicas, picking index 1
    T = it.RandomAffineWithInverse(degrees=15, scale=(0.8, 1.0), translate=(0.25, 0.25))
    torch.manual_seed(7)
    img = torch.from_numpy(recipes.uniform(43, (2, 3, 64, 64)))
    warped = T(img)
    theta = T.last_params["theta"]
    out["img"] = _np(img)
    out["theta"] = _np(theta)
    out["warped"] = _np(warped)
    A.grad = None
    At.grad = None
    l = opt.equivariance_loss(A, At[None].repeat(2, 1, 1, 1), T, 1)
    l.backward()
    out["equiv"] = _np(l)
    out["dA_equiv"] = _np(A.grad)
    out["dAt_equiv"] = _np(At.grad)
    out["inv_At"] = _np(T.inverse(At.detach()[None].repeat(2, 1, 1, 1)))
    # theta draw semantics (invertable_transform.py:42-57): seeded draws
    T2 = it.RandomAffineWithInverse(degrees=30, scale=(0.9, 1.1), translate=(0.1, 0.1))
    torch.manual_seed(123)
    T2(torch.zeros(3, 1, 4, 4))
    out["theta_seed123"] = _np(T2.last_params["theta"])
    np.savez_compressed(os.path.join(HERE, "losses.npz"), **out)


class _RecordingScheduler:
    def __init__(self, inner):
        self.inner = inner
        self.timesteps = inner.timesteps
        self.noises = []

    def add_noise(self, x, noise, t):
        self.noises.append(noise.clone())
        return self.inner.add_noise(x, noise, t)


def gen_step_tiny():
    """One token-opt micro-iteration (optimize.py:362-445) on the tiny SD-1.5-shaped model, CPU."""
    pu, opt = REFM.ptp_utils, REFM.optimize
    it = REFM.invertable_transform
    from stablekeypoints_amd.sd import build_sd15, TINY_CONFIG, TINY_IMAGE
    parts = build_sd15(seed=0, config=TINY_CONFIG)
    psum = float(sum(p.double().sum() for p in list(parts.unet.parameters()) + list(parts.vae.parameters())))
    parts.scheduler = _RecordingScheduler(parts.scheduler)
    latents = []
    enc = parts.vae.encode

    def recording_encode(x, *a, **k):   # record image2latent's VAE output (ptp_utils.py:300-303)
        out = enc(x, *a, **k)
        latents.append(out["latent_dist"].mean.detach().clone() * 0.18215)
        return out
    parts.vae.encode = recording_encode
    R, N = 32, 16
    controllers = {torch.device("cpu"): pu.AttentionStore()}

    def hook_fn(module, inp):   # optimize_token.py:59-68
        pu.register_attention_control(module, controllers[inp[0].device], feature_upsample_res=R)
    parts.unet.register_forward_pre_hook(hook_fn)
    img = torch.from_numpy(recipes.uniform(51, (1, 3, TINY_IMAGE, TINY_IMAGE)))
    ctx = torch.from_numpy(recipes.random_logits(52, (1, N, 32))).requires_grad_(True)
    T = it.RandomAffineWithInverse(degrees=15, scale=(0.8, 1.0), translate=(0.25, 0.25))
    kw = dict(layers=[0, 1, 2, 3], noise_level=-1, from_where=["down_cross", "mid_cross", "up_cross"],
              upsample_res=-1, device="cpu", controllers=controllers)
    torch.manual_seed(100)
    maps = pu.run_and_find_attn(parts, img, ctx, **kw)
    torch.manual_seed(101)
    timg = T(img)
    torch.manual_seed(102)
    maps_t = pu.run_and_find_attn(parts, timg, ctx, **kw)
    sigma, top_k, fps_n, bs, num_gpus = 2.0, 4, 8, 4, 1
    cand = pu.find_top_k_gaussian(maps[0], fps_n, sigma=sigma, num_subjects=1)
    idx = pu.furthest_point_sampling(maps_t[0], top_k, cand)
    sharp = opt.sharpening_loss(maps[0][idx], device="cpu", sigma=sigma, num_subjects=1)
    eq = opt.equivariance_loss(maps[0][idx], maps_t[0][idx][None].repeat(num_gpus, 1, 1, 1), T, 0)
    loss = (eq * 1000.0 + sharp * 100.0) / (bs // num_gpus)
    loss.backward()
    out = {"R": R, "N": N, "param_sum": psum, "img": _np(img), "ctx": _np(ctx), "timg": _np(timg),
           "theta": _np(T.last_params["theta"]), "noise0": _np(parts.scheduler.noises[0]),
           "noise1": _np(parts.scheduler.noises[1]), "latent0": _np(latents[0]), "latent1": _np(latents[1]),
           "map": _np(maps[0]), "map_t": _np(maps_t[0]),
           "cand": _np(cand), "idx": _np(idx), "sharp": _np(sharp), "eq": _np(eq), "loss": _np(loss),
           "dctx": _np(ctx.grad)}
    np.savez_compressed(os.path.join(HERE, "step_tiny.npz"), **out)


class _RecordingVAE:
    """Wraps vae.encode to record image2latent's latents (ptp_utils.py:300-303)."""

    def __init__(self, parts):
        self.latents = []
        enc = parts.vae.encode

        def recording_encode(x, *a, **k):
            out = enc(x, *a, **k)
            self.latents.append(out["latent_dist"].mean.detach().clone() * 0.18215)
            return out
        parts.vae.encode = recording_encode


def _tiny_parts_with_store(R):
    pu = REFM.ptp_utils
    from stablekeypoints_amd.sd import build_sd15, TINY_CONFIG
    parts = build_sd15(seed=0, config=TINY_CONFIG)
    parts.scheduler = _RecordingScheduler(parts.scheduler)
    rec = _RecordingVAE(parts)
    controllers = {torch.device("cpu"): pu.AttentionStore()}

    def hook_fn(module, inp):   # optimize_token.py:59-68
        pu.register_attention_control(module, controllers[inp[0].device], feature_upsample_res=R)
    parts.unet.register_forward_pre_hook(hook_fn)
    return parts, rec, controllers


class _cuda_as_cpu:
    """The reference hard-codes CUDA devices on its CPU-unreachable paths (eval.py:260, 473;
    keypoint_regressor.py:84 calls run_and_find_attn without a device, default "cuda").  For
    these CPU runs ``Tensor.to("cuda…")`` maps to "cpu" and ``Tensor.cuda()`` is the identity;
    nothing else changes."""

    def __enter__(self):
        self.orig = orig = torch.Tensor.to
        self.orig_cuda = torch.Tensor.cuda

        def to_cpu(t, *a, **k):
            if a and isinstance(a[0], str) and a[0].startswith("cuda"):
                a = ("cpu",) + a[1:]
            return orig(t, *a, **k)
        torch.Tensor.to = to_cpu
        torch.Tensor.cuda = lambda t, *a, **k: t   # eval.py:473 `.cuda()`

    def __exit__(self, *exc):
        torch.Tensor.to = self.orig
        torch.Tensor.cuda = self.orig_cuda


def gen_eval_tiny():
    """A15 run_image_with_context_augmented (eval.py:197-355) + find_max_pixel, tiny model, CPU.

    Thetas, VAE latents and noises of every augmentation are recorded so the GPU test can
    replay identical inputs.
    """
    ev, it = REFM.eval, REFM.invertable_transform
    from stablekeypoints_amd.sd import TINY_IMAGE
    R, N, S = 32, 16, 64
    parts, rec, controllers = _tiny_parts_with_store(R)
    thetas = []

    class RecAffine(it.RandomAffineWithInverse):
        def __call__(self, img_tensor, theta=None):
            out = super().__call__(img_tensor, theta)
            thetas.append(self.last_params["theta"].clone())
            return out
    ev.RandomAffineWithInverse = RecAffine
    img = torch.from_numpy(recipes.uniform(71, (3, TINY_IMAGE, TINY_IMAGE)))
    ctx = torch.from_numpy(recipes.random_logits(72, (1, N, 32)))
    indices = torch.tensor([3, 7, 0, 12, 5])
    with _cuda_as_cpu():
        torch.manual_seed(200)
        maps = ev.run_image_with_context_augmented(
            parts, img, ctx, indices, device="cpu", layers=[0, 1, 2, 3], augmentation_iterations=3, noise_level=-1,
            augment_degrees=30, augment_scale=(0.9, 1.1), augment_translate=(0.1, 0.1), controllers=controllers,
            num_gpus=1, upscale_size=S)
    kp = ev.find_max_pixel(maps.clone()) / float(S)
    out = {"R": R, "N": N, "S": S, "img_sha": recipes.sha256(_np(img)), "ctx": _np(ctx), "indices": _np(indices),
           "thetas": np.stack([_np(t) for t in thetas]), "noises": np.stack([_np(n) for n in parts.scheduler.noises]),
           "latents": np.stack([_np(l) for l in rec.latents]), "maps": _np(maps), "kp": _np(kp)}
    np.savez_compressed(os.path.join(HERE, "eval_tiny.npz"), **out)


def gen_best_indices_tiny():
    """keypoint_regressor.find_best_indices (keypoint_regressor.py:16-121), tiny model, CPU.

    The reference's "custom" dataset class is replaced by an in-memory one (its torchvision
    transforms are absent here); the DataLoader shuffle, the per-image capture, top-k, FPS and
    the unique/count ranking are the reference's own code.  Image order, latents and noises
    are recorded for the GPU replay.
    """
    kr = REFM.keypoint_regressor
    from stablekeypoints_amd.sd import TINY_IMAGE
    R, N, S = 32, 16, 32
    out = {"R": R, "N": N, "S": S}
    imgs = torch.from_numpy(recipes.uniform(81, (6, 3, TINY_IMAGE, TINY_IMAGE)))
    out["imgs_sha"] = recipes.sha256(_np(imgs))
    # The per-image maps are recorded too: the random-init tiny model's maps are flat, so the
    # argmax behind each Gaussian target (and hence the KL ranking) is decided by near-ties that
    # a 1e-6 map difference can flip.  The GPU test checks the maps to tolerance and every later
    # stage bit-exactly on the reference's own maps.  The "entropy" strategy is not pinned:
    # softmax over [0, 1]-valued maps is near-uniform for ANY input, so its ranking sits at fp32
    # summation noise (its kernel is checked against the fp64 oracle in test_gpu_parity).
    ctx = torch.from_numpy(recipes.random_logits(82, (1, N, 32)))
    out["ctx"] = _np(ctx)
    for strat in ("gaussian", "consistent"):
        parts, rec, controllers = _tiny_parts_with_store(R)
        parts.vae = types.SimpleNamespace(module=parts.vae)   # the device="cuda" branch reads vae.module
        order = []

        class MemDS(torch.utils.data.Dataset):
            def __init__(self, data_root=None, image_size=None):
                pass

            def __getitem__(self, i):
                order.append(i)
                return {"img": imgs[i], "kpts": torch.zeros(15, 2), "visibility": torch.zeros(15)}

            def __len__(self):
                return imgs.shape[0]
        kr.custom_images.CustomDataset = MemDS
        cands, picks = [], []
        pu = REFM.ptp_utils
        spy_fps, spy_topk = pu.furthest_point_sampling, pu.find_top_k_gaussian

        maps_seen = []

        def fps(maps, top_k, cand):
            maps_seen.append(maps.clone())
            cands.append(torch.as_tensor(cand).clone())
            out = spy_fps(maps, top_k, cand)
            picks.append(out.clone())
            return out
        pu.furthest_point_sampling = fps
        with _cuda_as_cpu():
            torch.manual_seed(300)
            idx = kr.find_best_indices(parts, ctx, num_steps=5, device="cpu", noise_level=-1, upsample_res=S,
                                       layers=[0, 1, 2, 3], top_k=4, dataset_name="custom",
                                       furthest_point_num_samples=8, controllers=controllers, num_gpus=1,
                                       top_k_strategy=strat, sigma=2.0)
        out[f"{strat}_order"] = np.array(order)
        out[f"{strat}_latents"] = np.stack([_np(l) for l in rec.latents])
        out[f"{strat}_noises"] = np.stack([_np(n) for n in parts.scheduler.noises])
        pu.furthest_point_sampling = spy_fps
        out[f"{strat}_indices"] = _np(idx)
        out[f"{strat}_cands"] = np.stack([_np(c) for c in cands])
        out[f"{strat}_picks"] = np.stack([_np(c) for c in picks])
        out[f"{strat}_maps"] = np.stack([_np(m) for m in maps_seen])
    np.savez_compressed(os.path.join(HERE, "best_indices_tiny.npz"), **out)


def gen_regressor():
    """keypoint_regressor.return_regressor / return_regressor_visible (:227-256), numpy."""
    kr = REFM.keypoint_regressor
    X = recipes.uniform(101, (40, 20)).astype(np.float64)
    Y = recipes.uniform(102, (40, 30)).astype(np.float64)
    vis = (recipes.uniform(103, (40, 30)) > 0.2).astype(np.float64)
    np.savez_compressed(os.path.join(HERE, "regressor.npz"), X=X, Y=Y, vis=vis, W=kr.return_regressor(X, Y),
                        Wv=kr.return_regressor_visible(X, Y, vis))


def gen_celeba_reader():
    """datasets/celeba.py:8-150 on a seeded 6-image tree (recipes.write_mini_celeba)."""
    import tempfile
    from datasets import celeba
    out = {}
    with tempfile.TemporaryDirectory() as root:
        recipes.write_mini_celeba(root)
        for align in (True, False):
            for split in ("train", "test"):
                ds = celeba.CelebA(split=split, align=align, dataset_loc=root)
                key = f"{'align' if align else 'wild'}_{split}"
                out[key + "_len"] = len(ds)
                out[key + "_img_sha"] = np.array([recipes.sha256(_np(ds[i]["img"])) for i in range(len(ds))])
                out[key + "_kpts"] = np.stack([_np(ds[i]["kpts"]) for i in range(len(ds))])
    np.savez_compressed(os.path.join(HERE, "celeba_reader.npz"), **out)


def gen_cub_reader():
    """datasets/cub_parts.py:242-440 (CUBDataset) on a seeded 6-image tree (recipes.write_mini_cub):
    train (jitter + mirror, np.random seeded per item) and test splits, cub_001 / cub_all.  The
    reference reader needs cv2.resize and torchvision's ToTensor, both absent here: they are
    supplied as restatements (cv2 INTER_LINEAR half-pixel bilinear / INTER_NEAREST floor, from
    stablekeypoints_amd.datasets; ToTensor = HWC uint8 -> CHW / 255), so the image pixels pin
    the crop, bbox padding/jitter, squaring and mirroring but not cv2's own resampling; the
    keypoints, visibility and sfm poses involve no resampling and are pinned outright."""
    import tempfile
    from datasets import cub_parts
    from stablekeypoints_amd import datasets as mine
    cv2 = sys.modules["cv2"]
    cv2.INTER_NEAREST = "nearest"

    def resize(img, size, interpolation=None):
        w, h = size
        if interpolation == "nearest":
            out = mine._resize_nearest(img[:, :, 0] if img.ndim == 3 else img, h, w)
        else:
            out = mine._resize_linear(img, h, w)
        return out

    cv2.resize = resize

    class _ToTensor:
        def __call__(self, im):
            a = np.asarray(im)
            return torch.from_numpy(a.transpose(2, 0, 1).copy()).float() / 255.0

    cub_parts.transforms = types.SimpleNamespace(Compose=lambda ts: ts[0], ToTensor=_ToTensor)
    out = {}
    with tempfile.TemporaryDirectory() as root:
        recipes.write_mini_cub(root)
        for split in ("train", "test"):
            for name, cls in (("001", 1), ("all", None)):
                ds = cub_parts.CUBDataset(dataset_root=root, split=split, single_class=cls)
                key = f"{split}_{name}"
                out[key + "_len"] = len(ds)
                out[key + "_labels"] = np.array(ds.labels)
                for i in range(len(ds)):
                    np.random.seed(100 + i)
                    e = ds[i]
                    out[f"{key}_{i}_img_sha"] = recipes.sha256(_np(e["img"]).astype(np.float32))
                    out[f"{key}_{i}_img_shape"] = np.array(e["img"].shape)
                    out[f"{key}_{i}_kpts"] = _np(e["kpts"])
                    out[f"{key}_{i}_vis"] = _np(e["visibility"])
                    out[f"{key}_{i}_mask_sha"] = recipes.sha256(np.asarray(e["mask"], np.float32))
                    out[f"{key}_{i}_sfm"] = np.asarray(e["sfm_pose"], np.float64)
    np.savez_compressed(os.path.join(HERE, "cub_reader.npz"), **out)


def gen_evaluate_tiny():
    """eval.evaluate (eval.py:374-539) on the tiny model, all five metrics, CPU.

    The test split is an in-memory 3-image set patched in for the CelebA class; per metric the
    reference's per-image maxima (find_max_pixel output), ground truth, errors (all_errors.pt)
    and, for inter_eye_distance, the replay inputs (thetas, latents, noises) are recorded.
    """
    import tempfile
    ev, it = REFM.eval, REFM.invertable_transform
    from stablekeypoints_amd.sd import TINY_IMAGE
    R, N, K = 32, 16, 32
    imgs = torch.from_numpy(recipes.uniform(111, (3, 3, TINY_IMAGE, TINY_IMAGE)))
    kpts = torch.from_numpy(recipes.uniform(112, (3, K, 2)))
    vis = torch.from_numpy((recipes.uniform(113, (3, K)) > 0.3).astype(np.float32))
    ctx = torch.from_numpy(recipes.random_logits(114, (1, N, 32)))
    indices = torch.tensor([2, 9, 14])
    W = torch.from_numpy(recipes.random_logits(115, (2 * len(indices), 2 * K), scale=0.3))
    out = {"R": R, "N": N, "imgs_sha": recipes.sha256(_np(imgs)), "kpts": _np(kpts), "vis": _np(vis),
           "ctx": _np(ctx), "indices": _np(indices), "W": _np(W)}
    for method in ("inter_eye_distance", "visible", "mean_average_error", "pck", "orientation_invariant"):
        parts, rec, controllers = _tiny_parts_with_store(R)
        order, highest, thetas = [], [], []

        class MemDS(torch.utils.data.Dataset):
            def __init__(self, *a, **k):
                pass

            def __getitem__(self, i):
                order.append(i)
                item = {"img": imgs[i], "kpts": kpts[i]}
                if method in ("visible", "mean_average_error"):
                    item["visibility"] = vis[i]
                return item

            def __len__(self):
                return imgs.shape[0]

        class RecAffine(it.RandomAffineWithInverse):
            def __call__(self, img_tensor, theta=None):
                o = super().__call__(img_tensor, theta)
                thetas.append(self.last_params["theta"].clone())
                return o
        spy_max = REFM.eval.find_max_pixel

        def find_max_pixel(maps):
            r = spy_max(maps)
            highest.append(r.clone())
            return r
        tta = ev.run_image_with_context_augmented

        def no_vis(*a, **k):   # evaluate plots image 0 (visualize=(i==0), 512² only): a side output
            k["visualize"] = False
            return tta(*a, **k)
        ev.CelebA = MemDS
        ev.RandomAffineWithInverse = RecAffine
        ev.find_max_pixel = find_max_pixel
        ev.run_image_with_context_augmented = no_vis
        with tempfile.TemporaryDirectory() as d, _cuda_as_cpu():
            torch.manual_seed(400)
            ev.evaluate(parts, ctx, indices, W, device="cpu", layers=[0, 1, 2, 3], augmentation_iterations=2,
                        save_folder=d, dataset_name="celeba_aligned", evaluation_method=method,
                        controllers=controllers, num_gpus=1)
            errs = torch.load(os.path.join(d, "all_errors.pt"), weights_only=True)
        ev.find_max_pixel = spy_max
        ev.run_image_with_context_augmented = tta
        out[f"{method}_order"] = np.array(order)
        out[f"{method}_highest"] = np.stack([_np(h) for h in highest])
        out[f"{method}_errors"] = _np(errs)
        if method == "inter_eye_distance":
            out["thetas"] = np.stack([_np(t) for t in thetas])
            out["latents"] = np.stack([_np(x) for x in rec.latents])
            out["noises"] = np.stack([_np(x) for x in parts.scheduler.noises])
    np.savez_compressed(os.path.join(HERE, "evaluate_tiny.npz"), **out)


def gen_theta_inv():
    """The reference's own θ⁻¹ (invertable_transform.py:72-92): the 2×3 matrix its ``inverse``
    hands to F.affine_grid, recorded by wrapping affine_grid, for seeded draws at the training
    augmentation (main.py:160-180: 15°, scale [0.8, 1], translate 0.25) and the TTA one
    (eval.py:224-228 defaults: 30°, [0.9, 1.1], 0.1), plus the inverse-warped image."""
    it = REFM.invertable_transform
    seen = []
    orig = it.F.affine_grid

    def rec(theta, size, align_corners=None):
        seen.append(theta.detach().clone())
        return orig(theta, size, align_corners=align_corners)
    it.F.affine_grid = rec
    out = {}
    try:
        for name, (deg, sc, tr) in (("train", (15, (0.8, 1.0), (0.25, 0.25))),
                                     ("tta", (30, (0.9, 1.1), (0.1, 0.1)))):
            T = it.RandomAffineWithInverse(degrees=deg, scale=sc, translate=tr)
            torch.manual_seed(500 if name == "train" else 501)
            img = torch.from_numpy(recipes.uniform(502, (64, 2, 24, 24)))
            seen.clear()
            T(img)
            theta = T.last_params["theta"].clone()
            inv_img = T.inverse(img)
            out[f"{name}_theta"] = _np(theta)
            out[f"{name}_theta_inv"] = _np(seen[1])
            out[f"{name}_inv_img"] = _np(inv_img)
        out["img"] = recipes.uniform(502, (64, 2, 24, 24))
    finally:
        it.F.affine_grid = orig
    np.savez_compressed(os.path.join(HERE, "theta_inv.npz"), **out)


def gen_entropy_ref():
    """The reference's fp32 Categorical entropies behind entropy_sort (ptp_utils.py:179-185) on the
    select golden's raw maps, recorded by wrapping the ``dist.Categorical`` it builds, plus the
    ranking torch.argsort gives them: exact fp32 ties at the top-25 boundary are ordered by
    torch's unspecified sort order."""
    pu = REFM.ptp_utils
    rec = []
    orig = pu.dist.Categorical

    class RecCat(orig):
        def entropy(self):
            e = super().entropy()
            rec.append(e.detach().clone())
            return e
    pu.dist.Categorical = RecCat
    try:
        maps = torch.from_numpy(recipes.attention_like_maps(31, 500, 128))
        order = pu.entropy_sort(maps, 25)
    finally:
        pu.dist.Categorical = orig
    np.savez_compressed(os.path.join(HERE, "entropy_ref.npz"), entropy_f32=_np(rec[0]), entropy25=_np(order))


def gen_sdxl_store():
    """The reference's SDXL-era AttentionStore (sdxl_monkey_patch.py:8-86, plain torch) driven by
    recipes.sdxl_store_scenario: returned tensors, counters, per-place stores, averages."""
    from unsupervised_keypoints import sdxl_monkey_patch as sm
    assert os.path.abspath(sm.__file__).startswith(REF), sm.__file__
    np.savez_compressed(os.path.join(HERE, "sdxl_store.npz"), **recipes.sdxl_store_scenario(sm.AttentionStore))


def gen_interp():
    """Torch interpolation/warp numerics the kernels restate."""
    import torch.nn.functional as F
    out = {}
    z = torch.from_numpy(recipes.random_logits(61, (3, 5, 6, 6)))
    out["z"] = _np(z)
    out["bicubic_6_to_32"] = _np(F.interpolate(z, size=(32, 32), mode="bicubic", align_corners=False))
    out["bicubic_6_to_13"] = _np(F.interpolate(z, size=(13, 13), mode="bicubic", align_corners=False))
    m = torch.from_numpy(recipes.random_logits(62, (1, 4, 16, 16)))
    out["m"] = _np(m)
    out["bilinear_16_to_40"] = _np(F.interpolate(m, size=(40, 40), mode="bilinear", align_corners=False))
    out["bilinear_16_to_64"] = _np(F.interpolate(m, size=(64, 64), mode="bilinear", align_corners=False))
    np.savez_compressed(os.path.join(HERE, "interp.npz"), **out)


if __name__ == "__main__":
    REFM = import_reference()
    torch.set_num_threads(8)
    which = sys.argv[1:] or ["capture_small", "capture_sd15", "argmax", "gaussian", "select", "losses",
                             "step_tiny", "interp", "eval_tiny", "best_indices_tiny", "regressor", "celeba_reader", "evaluate_tiny",
                             "cub_reader", "theta_inv", "entropy_ref", "sdxl_store"]
    for w in which:
        print("generating", w, flush=True)
        globals()["gen_" + w]()
