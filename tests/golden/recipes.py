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
