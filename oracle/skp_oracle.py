"""CPU oracle: numpy restatement of StableKeypoints' hot path (TEST INFRASTRUCTURE ONLY).

This module is the checker, never the product.  Only ``tests/``,
``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may import it;
``stablekeypoints_amd`` never does, and its ops fail loudly when the HIP library is
missing instead of falling back here.

Parity pinning: every function below is checked against golden vectors produced
by importing the reference itself in the build container
(``tests/golden/make_goldens.py``; fixtures ``tests/golden/*.npz``), see
``tests/test_oracle_golden.py``.  Each function cites the reference file:line
(paths relative to damaggu/StableKeypoints) it restates; torch semantics the
reference relies on are restated from SURVEY.md Appendix A.

Conventions: maps are float32 ``(T, h, w)``; positions are float32 ``(row, col)``
pixel centres (``index + 0.5``); indices are int64.
"""
import numpy as np

F32 = np.float32
A_CUBIC = -0.75  # torch upsample_bicubic2d Keys coefficient


# ----------------------------------------------------------------------------- interpolation
def _cubic_weights(t):
    """Keys cubic convolution weights for taps floor(src)-1 .. floor(src)+2 (A = -0.75)."""
    A = A_CUBIC

    def c1(x):  # |x| <= 1
        return ((A + 2) * x - (A + 3)) * x * x + 1

    def c2(x):  # 1 < |x| < 2
        return ((A * x - 5 * A) * x + 8 * A) * x - 4 * A
    return np.stack([c2(t + 1.0), c1(t), c1(1.0 - t), c2(2.0 - t)], axis=-1)


def bicubic_matrix(n_in, n_out):
    """(n_out, n_in) matrix of F.interpolate(mode="bicubic", align_corners=False) along one axis.

    src = (dst + 0.5) * n_in / n_out - 0.5 (not clamped for cubic); taps clamped to
    [0, n_in - 1] (used by ptp_utils.py:520-526).
    """
    scale = np.float32(n_in) / np.float32(n_out)
    dst = np.arange(n_out, dtype=np.float32)
    src = (dst + F32(0.5)) * scale - F32(0.5)
    i0 = np.floor(src).astype(np.int64)
    t = (src - i0).astype(np.float32)
    w = _cubic_weights(t).astype(np.float32)
    M = np.zeros((n_out, n_in), np.float32)
    for k in range(4):
        idx = np.clip(i0 - 1 + k, 0, n_in - 1)
        np.add.at(M, (np.arange(n_out), idx), w[:, k])
    return M


def bilinear_matrix(n_in, n_out):
    """(n_out, n_in) matrix of F.interpolate(mode="bilinear", align_corners=False) along one axis.

    src = max((dst + 0.5) * n_in / n_out - 0.5, 0); upper neighbour clamped
    (used by optimize.py:63-70).
    """
    scale = np.float32(n_in) / np.float32(n_out)
    dst = np.arange(n_out, dtype=np.float32)
    src = np.maximum((dst + F32(0.5)) * scale - F32(0.5), F32(0.0))
    i0 = src.astype(np.int64)
    i1 = np.minimum(i0 + 1, n_in - 1)
    l1 = (src - i0).astype(np.float32)
    l0 = F32(1.0) - l1
    M = np.zeros((n_out, n_in), np.float32)
    np.add.at(M, (np.arange(n_out), i0), l0)
    np.add.at(M, (np.arange(n_out), i1), l1)
    return M


def resize(x, n_out, kind):
    """Separable resize of the last two axes (square) with a bicubic/bilinear matrix."""
    n_in = x.shape[-1]
    M = bicubic_matrix(n_in, n_out) if kind == "bicubic" else bilinear_matrix(n_in, n_out)
    return np.einsum("yi,...ij,xj->...yx", M, x.astype(np.float32), M, optimize=True).astype(np.float32)


def resize_adjoint(g, n_in, kind):
    n_out = g.shape[-1]
    M = bicubic_matrix(n_in, n_out) if kind == "bicubic" else bilinear_matrix(n_in, n_out)
    return np.einsum("yi,...yx,xj->...ij", M, g.astype(np.float32), M, optimize=True).astype(np.float32)


# ----------------------------------------------------------------------------- A1 capture
def capture_fwd(z_low, s, R):
    """Captured attention of one layer from its low-resolution logits.

    Reference ptp_utils.py:513-536 computes softmax(to_q(bicubic(x)) kᵀ · scale).
    bicubic and to_q are linear and commute with ·kᵀ, so with
    z_low = (x W_qᵀ)_h k_hᵀ · scale  (the normal-path ``sim``, ptp_utils.py:493)
    attn_h = softmax_N(bicubic_{s→R}(z_low_h)).
    z_low: (H, s*s, N) -> attn (H, R*R, N).
    """
    H, S, N = z_low.shape
    z = z_low.reshape(H, s, s, N).transpose(0, 3, 1, 2)          # (H, N, s, s)
    Z = resize(z, R, "bicubic").transpose(0, 2, 3, 1).reshape(H, R * R, N)
    Z = Z - Z.max(axis=-1, keepdims=True)
    e = np.exp(Z)
    return (e / e.sum(axis=-1, keepdims=True)).astype(np.float32)


def capture_bwd(z_low, s, R, dattn):
    """d z_low from d attn (H, R*R, N): softmax backward then bicubic adjoint."""
    H, S, N = z_low.shape
    a = capture_fwd(z_low, s, R)
    dZ = a * (dattn - (a * dattn).sum(axis=-1, keepdims=True))
    dZ = dZ.reshape(H, R, R, N).transpose(0, 3, 1, 2)
    dz = resize_adjoint(dZ, s, "bicubic")                        # (H, N, s, s)
    return dz.transpose(0, 2, 3, 1).reshape(H, S, N).astype(np.float32)


def capture_maps_bwd_sel(z_layers, sizes, B, H, R, tok, gsel, gscale, heads=None):
    """d z_low of every captured layer for a SPARSE per-image map gradient (the
    skp_capture_maps_bwd_sel contract): image b's map gradient is gsel[b, k] (R*R) at token
    tok[b, k] (-1 = unused; duplicates add), zero elsewhere — the gradient the reference's
    losses produce, which read only maps[top_embedding_indices] (optimize.py:403-424) — scaled
    by gscale (1/(L*H): collect_maps' mean, optimize.py:75), broadcast over the image's H heads,
    then capture_bwd per head.  ``heads``: optional list of (b*H + h) rows to compute (the
    full-size tests check a subset).  Returns per layer (len(rows), s*s, N)."""
    N = z_layers[0].shape[-1]
    rows = list(range(B * H)) if heads is None else list(heads)
    out = []
    dense = np.zeros((B, N, R * R), np.float32)
    for b in range(B):
        for k in range(tok.shape[1]):
            if tok[b, k] >= 0:
                dense[b, tok[b, k]] += gsel[b, k].reshape(R * R)
    for z, s in zip(z_layers, sizes):
        res = []
        for bh in rows:
            g = (dense[bh // H] * F32(gscale)).T[None]             # (1, R*R, N)
            res.append(capture_bwd(z[bh:bh + 1], s, R, g)[0])
        out.append(np.stack(res))
    return out


def heads_split(t, H):
    """(B, S, H*d) -> (B*H, S, d) — CrossAttention.reshape_heads_to_batch_dim (diffusers 0.8.0)."""
    b, s, hd = t.shape
    return t.reshape(b, s, H, hd // H).transpose(0, 2, 1, 3).reshape(b * H, s, hd // H)


def heads_merge(t, H):
    bh, s, d = t.shape
    return t.reshape(bh // H, H, s, d).transpose(0, 2, 1, 3).reshape(bh // H, s, d * H)


def cross_attn_logits(x, ctx, Wq, Wk, H):
    """z_low = (x Wqᵀ)(ctx Wkᵀ)ᵀ · d^-½ per head (ptp_utils.py:483-493)."""
    q = heads_split(x @ Wq.T, H)
    k = heads_split(ctx @ Wk.T, H)
    scale = F32((Wq.shape[0] // H) ** -0.5)
    return (q @ k.transpose(0, 2, 1) * scale).astype(np.float32), q, k, scale


def cross_attn_logits_bwd(dz, q, k, scale, x, ctx, Wq, Wk, H):
    dq = heads_merge(dz @ k * scale, H)
    dk = heads_merge(dz.transpose(0, 2, 1) @ q * scale, H)
    return (dq @ Wq).astype(np.float32), (dk @ Wk).astype(np.float32)


# ----------------------------------------------------------------------------- A3 aggregate
def collect_maps(attn_layers, layers=(0, 1, 2, 3), upsample_res=-1, indices=None):
    """optimize.collect_maps (optimize.py:27-79): per layer (B·H, R², N) -> mean (N', R', R').

    Layer selection by position (44-48), optional token gather (58-59), bilinear
    up-res when upsample_res != -1 (63-70; the size guard compares the token
    count, so it always fires), then mean over layers and B·heads (75).
    """
    acc = []
    for li, a in enumerate(attn_layers):
        if li not in layers:
            continue
        BH, S, N = a.shape
        R = int(round(S ** 0.5))
        d = a.reshape(BH, R, R, N)
        if indices is not None:
            d = d[..., np.asarray(indices)]
        d = d.transpose(0, 3, 1, 2)
        if upsample_res != -1 and d.shape[1] ** 0.5 != upsample_res:
            d = resize(d, upsample_res, "bilinear")
        acc.append(d.astype(np.float32))
    return np.stack(acc).mean(axis=(0, 1), dtype=np.float64).astype(np.float32)


def collect_maps_bwd(attn_shapes, dmap, layers=(0, 1, 2, 3), upsample_res=-1, indices=None):
    """Gradient of collect_maps w.r.t. each stored layer (broadcast mean, gather/bilinear adjoint)."""
    sel = [li for li in range(len(attn_shapes)) if li in layers]
    out = []
    for li, (BH, S, N) in enumerate(attn_shapes):
        if li not in sel:
            out.append(np.zeros((BH, S, N), np.float32))
            continue
        R = int(round(S ** 0.5))
        g = dmap / F32(len(sel) * BH)
        if upsample_res != -1 and R != upsample_res:
            g = resize_adjoint(g, R, "bilinear")
        full = np.zeros((N, R, R), np.float32)
        if indices is not None:
            np.add.at(full, np.asarray(indices), g)
        else:
            full = g
        out.append(np.broadcast_to(full.reshape(N, S).T[None], (BH, S, N)).astype(np.float32))
    return out


# ----------------------------------------------------------------------------- A4-A6 argmax
def _argmax_first_nan(flat):
    """torch.argmax semantics: first occurrence of the max; NaN counts as the maximum."""
    nan = np.isnan(flat)
    out = np.empty(flat.shape[0], np.int64)
    for i in range(flat.shape[0]):
        if nan[i].any():
            out[i] = int(np.argmax(nan[i]))
        else:
            out[i] = int(np.argmax(flat[i]))
    return out


def find_max_pixel(m):
    """eval.find_max_pixel (eval.py:39-60): (row, col) + 0.5 of the per-map argmax."""
    T, h, w = m.shape
    idx = _argmax_first_nan(m.reshape(T, -1))
    return (np.stack([idx // w, idx % w], axis=-1).astype(np.float32) + F32(0.5))


def mask_radius(m, max_coords, radius):
    """eval.mask_radius (eval.py:83-111): multiply by (squared distance > radius²)."""
    T, h, w = m.shape
    x = np.arange(w, dtype=np.float32)[None, None, :]
    y = np.arange(h, dtype=np.float32)[None, :, None]
    d2 = (x - max_coords[:, 1][:, None, None]) ** 2 + (y - max_coords[:, 0][:, None, None]) ** 2
    mask = (d2 > F32(radius ** 2)).astype(np.float32)
    with np.errstate(invalid="ignore"):
        return (m * mask).astype(np.float32)


def find_k_max_pixels(m, num=3):
    """eval.find_k_max_pixels (eval.py:62-81): num rounds of argmax + mask_radius(0.05·h)."""
    T, h, w = m.shape
    pts = []
    for _ in range(num):
        p = find_max_pixel(m)
        pts.append(p)
        m = mask_radius(m, p, 0.05 * h)
    return np.stack(pts)


def pixel_from_weighted_avg(m, distance=5):
    """eval.pixel_from_weighted_avg (eval.py:113-155); returns (pos, mutated map)."""
    m = m.copy()
    T, h, w = m.shape
    if distance != -1:
        p = find_max_pixel(m)
        r, c = p[:, 0].astype(np.int64), p[:, 1].astype(np.int64)
        x = np.arange(h, dtype=np.float32)[None, :, None]
        y = np.arange(w, dtype=np.float32)[None, None, :]
        d = np.sqrt((x - r[:, None, None].astype(np.float32)) ** 2 + (y - c[:, None, None].astype(np.float32)) ** 2)
        m[d > distance] = 0.0
    tot = m.sum(axis=(1, 2), keepdims=True, dtype=np.float64).astype(np.float32)
    nm = m / (tot + F32(1e-6))
    x = np.arange(h, dtype=np.float32)[None, :, None]
    y = np.arange(w, dtype=np.float32)[None, None, :]
    xs = (x * nm).sum(axis=(1, 2), dtype=np.float64)
    ys = (y * nm).sum(axis=(1, 2), dtype=np.float64)
    return (np.stack([xs, ys], axis=-1) + 0.5).astype(np.float32), m


# ----------------------------------------------------------------------------- A7 target
def gaussian_circle(pos, size, sigma):
    """optimize_token.gaussian_circle (optimize_token.py:204-224); pos (T, 2) in [0,1] (row, col)."""
    p = pos.astype(np.float32) * F32(size)
    g = np.arange(size, dtype=np.float32) + F32(0.5)
    di = g[None, :, None] - p[:, 0][:, None, None]
    dj = g[None, None, :] - p[:, 1][:, None, None]
    d2 = dj * dj + di * di
    return np.exp(-d2 / F32(2.0 * sigma ** 2.0)).astype(np.float32)


def gaussian_circles(pos, size, sigma):
    """optimize_token.gaussian_circles (226-242): mean over subjects; pos (num, T, 2)."""
    return np.mean(np.stack([gaussian_circle(p, size, sigma) for p in pos]), axis=0, dtype=np.float32)


# ----------------------------------------------------------------------------- A8-A10 select
def kl_to_gaussian(m, sigma, epsilon=1e-5, num_subjects=1):
    """Per-token KL(target ‖ softmax(map)) of ptp_utils.find_top_k_gaussian (ptp_utils.py:86-108)."""
    T, h, w = m.shape
    pos = find_k_max_pixels(m, num=num_subjects) / F32(h)
    x = m.reshape(T, -1).astype(np.float32) + F32(epsilon)
    x = x - x.max(axis=-1, keepdims=True)
    e = np.exp(x)
    P = e / e.sum(axis=-1, keepdims=True, dtype=np.float64).astype(np.float32)
    tgt = gaussian_circles(pos, h, sigma).reshape(T, -1) + F32(epsilon)
    tgt = tgt / tgt.sum(axis=-1, keepdims=True, dtype=np.float64).astype(np.float32)
    return (tgt.astype(np.float64) * (np.log(tgt.astype(np.float64)) - np.log(P.astype(np.float64)))).sum(axis=-1)


def find_top_k_gaussian(m, top_k, sigma=3, epsilon=1e-5, num_subjects=1):
    """ptp_utils.find_top_k_gaussian (86-112): ascending KL, first top_k (stable tie policy)."""
    kl = kl_to_gaussian(m, sigma, epsilon, num_subjects)
    return np.argsort(kl, kind="stable")[:top_k].astype(np.int64)


def entropy_values(m):
    """Entropy of softmax(map) per token (ptp_utils.py:179-182), in fp64."""
    T = m.shape[0]
    x = m.reshape(T, -1).astype(np.float64)
    x = x - x.max(axis=-1, keepdims=True)
    lp = x - np.log(np.exp(x).sum(axis=-1, keepdims=True))
    return -(np.exp(lp) * lp).sum(axis=-1)


def entropy_sort(m, top_k):
    """ptp_utils.entropy_sort (165-187): ascending entropy of softmax(map), first top_k."""
    return np.argsort(entropy_values(m), kind="stable")[:top_k].astype(np.int64)


def _dist(a, b):
    d = (a - b).astype(np.float32)
    return np.float32(np.sqrt(np.float64((d * d).sum(axis=-1, dtype=np.float32))))


def furthest_point_sampling(m, top_k, cand):
    """ptp_utils.furthest_point_sampling (115-159): argmax positions, strict '>' first-wins."""
    T, h, w = m.shape
    pos = find_max_pixel(m) / F32(h)
    cand = [int(c) for c in cand]
    max_dist = -1.0
    pair = None
    for i in range(len(cand)):
        for j in range(i + 1, len(cand)):
            d = _dist(pos[cand[i]], pos[cand[j]])
            if d > max_dist:
                max_dist = d
                pair = (cand[i], cand[j])
    if pair is None:
        raise ValueError("furthest_point_sampling needs at least two candidates")
    sel = [pair[0], pair[1]]
    for _ in range(top_k - 2):
        best, best_i = -1.0, None
        for i in cand:
            if i in sel:
                continue
            dm = min(_dist(pos[i], pos[s]) for s in sel)
            if dm > best:
                best, best_i = dm, i
        if best_i is not None:
            sel.append(best_i)
    return np.asarray(sel, np.int64)


# ----------------------------------------------------------------------------- A11 sharpening
def sharpening_loss(A, sigma, num_subjects=1):
    """optimize.sharpening_loss (166-179) + find_gaussian_loss_at_point (182-206).

    Returns (loss, dloss/dA); the Gaussian target carries no gradient.
    """
    T, h, w = A.shape
    pos = find_k_max_pixels(A, num=num_subjects) / F32(w)
    G = gaussian_circles(pos, h, sigma)
    diff = (A - G).astype(np.float32)
    loss = np.float32((diff.astype(np.float64) ** 2).mean())
    return loss, (F32(2.0 / diff.size) * diff).astype(np.float32)


# ----------------------------------------------------------------------------- A12 warp
def affine_params(rng_uniforms, degrees, scale, translate):
    """theta draw of RandomAffineWithInverse.__call__ (invertable_transform.py:42-57, 22-36).

    ``rng_uniforms``: (B, 4) U[0,1) draws in the reference's order (angle, scale, tx, ty).
    """
    import math
    th = []
    for u in rng_uniforms:
        ang = float(u[0]) * (2 * degrees) - degrees
        sc = float(u[1]) * (scale[1] - scale[0]) + scale[0]
        tx = float(u[2]) * (2 * translate[0]) - translate[0]
        ty = float(u[3]) * (2 * translate[1]) - translate[1]
        a = math.radians(ang)
        t = np.array([[math.cos(a), math.sin(a), tx], [-math.sin(a), math.cos(a), ty]], np.float32)
        t[:, :2] = t[:, :2] * np.float32(sc)
        th.append(t)
    return np.stack(th).astype(np.float32)


def theta_inverse(theta):
    """RandomAffineWithInverse.inverse (72-84): 2x3 part of the 3x3 inverse, in the reference's
    arithmetic: fp32 ``torch.inverse`` (LU with partial pivoting through torch-CPU's LAPACK) of the
    fp32 3x3 batch.  numpy's float32 ``linalg.inv`` rounds differently (1 ulp on ≈25% of entries
    of tests/golden/theta_inv.npz), so this one call goes through torch-CPU, the reference's own
    arithmetic dependency: bit-identical to the reference's recorded θ⁻¹ on the golden's host, and
    to the reference on any other host (MKL's LU code path, and so the last bit, follows the CPU)."""
    import torch
    B = theta.shape[0]
    aug = np.concatenate([np.asarray(theta, np.float32), np.tile(np.array([[[0, 0, 1.0]]], np.float32), (B, 1, 1))],
                         axis=1)
    return torch.inverse(torch.from_numpy(aug))[:, :2, :].numpy().astype(np.float32)


def _fma32(a, b, c):
    """float32 fused multiply-add (the product is exact in float64)."""
    return (np.asarray(a, np.float64) * np.asarray(b, np.float64) + np.asarray(c, np.float64)).astype(np.float32)


def _base_coords(n):
    """affine_grid base coordinates, align_corners=False: linspace(-1,1,n)·(n-1)/n."""
    if n == 1:
        return np.zeros(1, np.float32)
    # torch-CPU linspace rounding (bit-equal to torch.linspace, tests/test_oracle_golden.py):
    # fma(i, step, -1) for the first half, fma(-(n-1-i), step, 1) for the second
    step = np.float32(np.float32(2.0) / np.float32(n - 1))
    i = np.arange(n)
    lin = np.where(i < n // 2, _fma32(i, step, -1.0), _fma32(-(n - 1 - i), step, 1.0)).astype(np.float32)
    return ((lin * np.float32(n - 1)) / np.float32(n)).astype(np.float32)


def _grid(theta, H, W):
    """Sampling coordinates of F.affine_grid + grid_sample as torch-CPU rounds them (the reference
    warps images on the CPU, optimize.py:386): the affine_grid bmm of [x, y, 1] by θᵀ as
    fma(y, θ1, x·θ0) + θ2 (bit-equal to F.affine_grid, checked in tests/test_oracle_golden.py) and
    the CPU grid sampler's unnormalisation fma(g + 1, n/2, −0.5)."""
    xs = _base_coords(W)[None, None, :]
    ys = _base_coords(H)[None, :, None]
    t = theta.astype(np.float32)
    gx = _fma32(ys, t[:, 0, 1, None, None], xs * t[:, 0, 0, None, None]) + t[:, 0, 2, None, None]
    gy = _fma32(ys, t[:, 1, 1, None, None], xs * t[:, 1, 0, None, None]) + t[:, 1, 2, None, None]
    ix = _fma32(gx + F32(1.0), F32(W / 2), -0.5)
    iy = _fma32(gy + F32(1.0), F32(H / 2), -0.5)
    return ix.astype(np.float32), iy.astype(np.float32)


def _taps(ix, iy, H, W):
    """grid_sample bilinear taps (nw, ne, sw, se) with the CPU sampler's weight formulas:
    w = ix − floor(ix), e = 1 − w, n = iy − floor(iy), s = 1 − n; nw = s·e, ne = s·w, sw = n·e,
    se = n·w (summed in that order by the callers)."""
    x0f = np.floor(ix).astype(np.float32)
    y0f = np.floor(iy).astype(np.float32)
    x1f, y1f = x0f + F32(1.0), y0f + F32(1.0)
    we = (ix - x0f).astype(np.float32)
    ee = (F32(1.0) - we).astype(np.float32)
    wn = (iy - y0f).astype(np.float32)
    ws = (F32(1.0) - wn).astype(np.float32)
    wts = [((y0f, x0f), ws * ee), ((y0f, x1f), ws * we), ((y1f, x0f), wn * ee), ((y1f, x1f), wn * we)]
    out = []
    for (yf, xf), w in wts:
        yy, xx = yf.astype(np.int64), xf.astype(np.int64)
        ok = (yy >= 0) & (yy < H) & (xx >= 0) & (xx < W)
        out.append((np.clip(yy, 0, H - 1), np.clip(xx, 0, W - 1), (w * ok).astype(np.float32)))
    return out


def affine_warp(img, theta):
    """F.grid_sample(img, F.affine_grid(theta), bilinear, zeros, align_corners=False)
    (invertable_transform.py:64-70, 86-90).  img (B, C, H, W), theta (B, 2, 3)."""
    B, C, H, W = img.shape
    ix, iy = _grid(theta, H, W)
    out = np.zeros_like(img, dtype=np.float32)
    for b in range(B):
        for yy, xx, w in _taps(ix[b], iy[b], H, W):
            out[b] += img[b][:, yy, xx] * w[None]
    return out


def affine_warp_bwd(gout, theta, H, W):
    """Adjoint of affine_warp w.r.t. its input (bilinear scatter-add)."""
    B, C = gout.shape[:2]
    ix, iy = _grid(theta, H, W)
    gin = np.zeros((B, C, H, W), np.float32)
    for b in range(B):
        for yy, xx, w in _taps(ix[b], iy[b], H, W):
            for c in range(C):
                np.add.at(gin[b, c], (yy, xx), gout[b, c] * w)
    return gin


def equivariance_loss(A, At, theta, index):
    """optimize.equivariance_loss (157-163) for the replica ``index``.

    The reference inverse-warps map_t repeated over all replicas and keeps row
    ``index``; only theta[index] matters.  Returns (loss, dA, dAt).
    """
    ti = theta_inverse(theta[index:index + 1])
    Ap = affine_warp(At[None], ti)[0]
    diff = (A - Ap).astype(np.float32)
    loss = np.float32((diff.astype(np.float64) ** 2).mean())
    g = (F32(2.0 / diff.size) * diff).astype(np.float32)
    dAt = affine_warp_bwd(-g[None], ti, A.shape[1], A.shape[2])[0]
    return loss, g, dAt
