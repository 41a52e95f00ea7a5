"""Deterministic input recipes shared by the golden generator and the tests.

Large inputs (e.g. 500 x 128 x 128 maps = 32.8 MB) are not committed; the
fixtures store the recipe parameters plus a SHA-256 of the generated array, and
the tests regenerate the array with these numpy-only (PCG64) recipes and check
the hash before trusting a comparison.
"""
import hashlib

import numpy as np


def sha256(a):
    a = np.ascontiguousarray(a)
    return hashlib.sha256(a.tobytes()).hexdigest()


def attention_like_maps(seed, n_tokens, size, n_layers_heads=1):
    """Maps that look like aggregated cross-attention: a bump per token + noise.

    Returns float32 (n_tokens, size, size) in [0, 1) with row sums over tokens
    close to 1 at every pixel (like a token softmax averaged over heads).
    """
    rng = np.random.default_rng(seed)
    yy, xx = np.meshgrid(np.arange(size), np.arange(size), indexing="ij")
    cy = rng.uniform(0, size, n_tokens)
    cx = rng.uniform(0, size, n_tokens)
    width = rng.uniform(0.03, 0.25, n_tokens) * size
    amp = rng.uniform(0.5, 4.0, n_tokens)
    logits = np.empty((n_tokens, size, size), np.float64)
    for t in range(n_tokens):
        d2 = (yy - cy[t]) ** 2 + (xx - cx[t]) ** 2
        logits[t] = amp[t] * np.exp(-d2 / (2 * width[t] ** 2))
    logits += rng.normal(0, 0.3, logits.shape)
    logits -= logits.max(axis=0, keepdims=True)
    p = np.exp(logits)
    p /= p.sum(axis=0, keepdims=True)
    return p.astype(np.float32)


def random_logits(seed, shape, scale=1.0):
    rng = np.random.default_rng(seed)
    return (rng.standard_normal(shape) * scale).astype(np.float32)


def uniform(seed, shape, lo=0.0, hi=1.0):
    rng = np.random.default_rng(seed)
    return rng.uniform(lo, hi, shape).astype(np.float32)


def argmax_edge_cases():
    """Small maps exercising ties, plateaus, NaN, inf, negatives (A4/A5/A6)."""
    cases = []
    m = np.zeros((4, 4), np.float32); m[1, 2] = 1.0; m[3, 0] = 1.0; cases.append(m)          # tie -> first
    m = np.ones((4, 4), np.float32); cases.append(m)                                         # all equal
    m = np.zeros((4, 4), np.float32); m[2, 2] = np.nan; m[0, 1] = 5.0; cases.append(m)       # NaN is max
    m = np.zeros((4, 4), np.float32); m[3, 3] = np.nan; m[1, 1] = np.nan; cases.append(m)    # first NaN
    m = -np.arange(16, dtype=np.float32).reshape(4, 4); cases.append(m)                     # negatives
    m = np.zeros((4, 4), np.float32); m[0, 3] = np.inf; m[2, 1] = np.inf; cases.append(m)    # inf tie
    m = np.full((4, 4), -np.inf, np.float32); cases.append(m)                               # all -inf
    m = np.zeros((4, 4), np.float32); m[3, 3] = 1e-30; cases.append(m)                       # tiny
    return np.stack(cases)


def cross_attention_params(seed, layer, c, ctx_dim):
    """Seeded parameters of one diffusers-0.8.0 CrossAttention(c, ctx_dim) in named_parameters order."""
    shapes = [("to_q.weight", (c, c)), ("to_k.weight", (c, ctx_dim)), ("to_v.weight", (c, ctx_dim)),
              ("to_out.0.weight", (c, c)), ("to_out.0.bias", (c,))]
    out = {}
    for pi, (name, shp) in enumerate(shapes):
        bound = 1.0 / np.sqrt(shp[-1])
        out[name] = uniform(seed * 100 + layer * 10 + pi, shp, -bound, bound)
    return out


def capture_inputs(seed, shapes, n_tokens, ctx_dim):
    """Layer inputs x_l (1, s*s, C), context (1, N, D) and per-layer CrossAttention params."""
    xs = [random_logits(seed * 7 + i, (1, s * s, c)) for i, (s, c) in enumerate(shapes)]
    ctx = random_logits(seed * 7 + 99, (1, n_tokens, ctx_dim))
    params = [cross_attention_params(seed, li, c, ctx_dim) for li, (s, c) in enumerate(shapes)]
    return xs, ctx, params


def write_mini_celeba(root, seed=0):
    """A 6-image CelebA tree (datasets/celeba.py layout) with seeded random pixels, sizes,
    landmarks and face boxes: aligned PNGs and in-the-wild JPEGs, MAFL train/test lists.
    Images 2 and 5 get face boxes below the wild reader's 30 % area threshold."""
    import os
    from PIL import Image
    rng = np.random.default_rng(seed)
    n = 6
    for sub in ("Anno", "MAFL", "Img/img_align_celeba_png", "Img/img_celeba"):
        os.makedirs(os.path.join(root, sub), exist_ok=True)
    lm_a, lm_w, bb = [f"{n}\n", "lefteye_x lefteye_y ...\n"], [f"{n}\n", "lefteye_x lefteye_y ...\n"], \
        [f"{n}\n", "image_id x_1 y_1 width height\n"]
    for k in range(n):
        name = f"{k + 1:06d}"
        ha, wa = int(rng.integers(40, 64)), int(rng.integers(40, 64))
        Image.fromarray(rng.integers(0, 256, (ha, wa, 3), dtype=np.uint8)).save(
            os.path.join(root, "Img/img_align_celeba_png", name + ".png"))
        hw, ww = int(rng.integers(48, 80)), int(rng.integers(48, 80))
        Image.fromarray(rng.integers(0, 256, (hw, ww, 3), dtype=np.uint8)).save(
            os.path.join(root, "Img/img_celeba", name + ".jpg"), quality=90)
        pa = rng.uniform(0, 1, (5, 2)) * [wa, ha]
        pw = rng.uniform(0, 1, (5, 2)) * [ww, hw]
        lm_a.append(name + ".jpg " + " ".join(str(int(v)) for v in pa.ravel()) + "\n")
        lm_w.append(name + ".jpg " + " ".join(str(int(v)) for v in pw.ravel()) + "\n")
        frac = 0.1 if k in (2, 5) else 0.6
        bw, bh = int(ww * np.sqrt(frac)), int(hw * np.sqrt(frac))
        bb.append(f"{name}.jpg 1 2 {bw} {bh}\n")
    open(os.path.join(root, "Anno/list_landmarks_align_celeba.txt"), "w").writelines(lm_a)
    open(os.path.join(root, "Anno/list_landmarks_celeba.txt"), "w").writelines(lm_w)
    open(os.path.join(root, "Anno/list_bbox_celeba.txt"), "w").writelines(bb)
    open(os.path.join(root, "MAFL/training.txt"), "w").writelines(["000001.jpg\n", "000003.jpg\n", "000004.jpg\n",
                                                                   "000006.jpg\n"])
    open(os.path.join(root, "MAFL/testing.txt"), "w").writelines(["000002.jpg\n", "000005.jpg\n"])


def write_mini_cub(root, seed=0):
    """A 6-image CUB tree in the layout datasets/cub_parts.py reads: PNG images (lossless, so the
    bytes the readers see are the seeded pixels; the reader only joins rel_path) under
    CUB_200_2011/images/<class dir>/, CMR-style train/test .mat annotations (struct array
    ``images``: rel_path, bbox x1..y2 1-based, parts 3 × 15 (x, y, visibility, 1-based), mask)
    and .../sfm/anno_<split>.mat (``sfm_anno``: scale, trans (2,), rot 3 × 3).  Classes 001 ×3,
    002 ×2, 003 ×1; image 1 is grayscale; image 4's box runs past the image (background fill)."""
    import os
    import scipy.io as sio
    from PIL import Image
    rng = np.random.default_rng(seed)
    classes = [1, 1, 2, 1, 2, 3]
    base = os.path.join(root, "CUB_200_2011")
    recs, sfms = [], []
    for k, c in enumerate(classes):
        d = f"{c:03d}.Bird_{c}"
        os.makedirs(os.path.join(base, "images", d), exist_ok=True)
        h, w = int(rng.integers(60, 100)), int(rng.integers(60, 100))
        shape = (h, w) if k == 1 else (h, w, 3)
        rel = f"{d}/Bird_{c}_{k:04d}.png"
        Image.fromarray(rng.integers(0, 256, shape, dtype=np.uint8)).save(os.path.join(base, "images", rel))
        x1, y1 = int(rng.integers(2, w // 3)), int(rng.integers(2, h // 3))
        x2 = w + 5 if k == 4 else int(rng.integers(2 * w // 3, w))
        y2 = int(rng.integers(2 * h // 3, h))
        parts = np.zeros((3, 15))
        parts[0] = rng.uniform(x1, min(x2, w), 15).round()
        parts[1] = rng.uniform(y1, y2, 15).round()
        parts[2] = (rng.uniform(0, 1, 15) > 0.3).astype(float)
        parts[:2, parts[2] == 0] = 0.0
        mask = (rng.uniform(0, 1, (h, w)) > 0.5).astype(np.uint8)
        recs.append((rel, {"x1": float(x1), "y1": float(y1), "x2": float(x2), "y2": float(y2)}, parts, mask))
        q = rng.normal(size=4)
        q /= np.linalg.norm(q)
        a, b_, c_, d_ = q
        rot = np.array([[1 - 2 * (c_ * c_ + d_ * d_), 2 * (b_ * c_ - a * d_), 2 * (b_ * d_ + a * c_)],
                        [2 * (b_ * c_ + a * d_), 1 - 2 * (b_ * b_ + d_ * d_), 2 * (c_ * d_ - a * b_)],
                        [2 * (b_ * d_ - a * c_), 2 * (c_ * d_ + a * b_), 1 - 2 * (b_ * b_ + c_ * c_)]])
        sfms.append((float(rng.uniform(50, 150)), rng.uniform(20, 60, 2), rot))
    cache = os.path.join(base, "cachedir", "cub")
    os.makedirs(os.path.join(cache, "data"), exist_ok=True)
    os.makedirs(os.path.join(cache, "sfm"), exist_ok=True)
    for split, idx in (("train", [0, 1, 2, 3, 4, 5]), ("test", [5, 2, 0, 4])):
        imgs = np.zeros((len(idx),), dtype=[("rel_path", "O"), ("bbox", "O"), ("parts", "O"), ("mask", "O")])
        sfm = np.zeros((len(idx),), dtype=[("scale", "O"), ("trans", "O"), ("rot", "O")])
        for j, k in enumerate(idx):
            imgs[j]["rel_path"], imgs[j]["bbox"], imgs[j]["parts"], imgs[j]["mask"] = recs[k]
            sfm[j]["scale"], sfm[j]["trans"], sfm[j]["rot"] = sfms[k]
        sio.savemat(os.path.join(cache, "data", f"{split}_cub_cleaned.mat"), {"images": imgs})
        sio.savemat(os.path.join(cache, "sfm", f"anno_{split}.mat"), {"sfm_anno": sfm})


# The SDXL store scenario (sdxl_monkey_patch.py:8-86): a sequence of attention-probability calls
# driven through an ``AttentionStore`` class (the reference's when the golden is made, this
# package's in the test), five layers per diffusion step, three steps, then a fourth step with a
# subclass that marks the first two layers unconditional.  Returns the numpy record the golden
# holds.  (shape, is_cross, place): 1024 pixels is kept (the 32² boundary), 1025 is not.
SDXL_STORE_CALLS = [((4, 1024, 7), True, "down"), ((4, 1025, 7), True, "up"), ((4, 64, 64), False, "mid"),
                    ((4, 256, 7), True, "up"), ((2, 16, 16), False, "down")]


def sdxl_store_scenario(store_cls):
    import torch
    out = {}

    def drive(ctl, steps, tag):
        for st in range(steps):
            for ci, (shape, is_cross, place) in enumerate(SDXL_STORE_CALLS):
                g = torch.Generator().manual_seed(1000 * st + ci + (7 if tag == "uncond" else 0))
                attn = torch.rand(shape, generator=g).softmax(dim=-1)
                ret = ctl(attn, is_cross, place)
                assert ret is attn
                if shape[1] <= 256:
                    out[f"{tag}_ret_{st}_{ci}"] = ret.numpy().copy()
            out[f"{tag}_counters_{st}"] = np.array([ctl.cur_step, ctl.cur_att_layer])
        for key, maps in ctl.attention_store.items():
            out[f"{tag}_nstore_{key}"] = np.array(len(maps))
            for i, m in enumerate(maps):
                out[f"{tag}_store_{key}_{i}"] = m.numpy().copy()
        for key, maps in ctl.get_average_attention().items():
            for i, m in enumerate(maps):
                out[f"{tag}_avg_{key}_{i}"] = m.numpy().copy()
        out[f"{tag}_keys"] = np.array(list(ctl.get_empty_store().keys()))

    ctl = store_cls()
    ctl.num_att_layers = len(SDXL_STORE_CALLS)
    drive(ctl, 3, "plain")
    ctl.reset()
    out["plain_after_reset"] = np.array([ctl.cur_step, ctl.cur_att_layer, len(ctl.attention_store),
                                         sum(len(v) for v in ctl.step_store.values())])

    class Uncond(store_cls):
        @property
        def num_uncond_att_layers(self):
            return 2

    ctl = Uncond()
    ctl.num_att_layers = len(SDXL_STORE_CALLS) - 2
    drive(ctl, 2, "uncond")
    return out
