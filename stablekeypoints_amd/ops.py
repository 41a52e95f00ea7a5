"""Torch-facing ops over libskp (HIP, gfx950): autograd Functions and plain wrappers.

Every function here launches the HIP kernels through the C ABI (``_lib``) on the
current HIP stream; there is no CPU or eager-torch fallback for the hot path.
"""
import ctypes
import os

import torch

from . import _lib
from ._lib import call, ptr, stream

F32 = torch.float32

# Optional per-kernel timer (bench.py): an object with record(name, nbytes) returning a
# context manager that brackets one launch with HIP events on the current stream.
_TIMER = None


def set_kernel_timer(timer):
    global _TIMER
    _TIMER = timer


class _NoTimer:
    def __enter__(self):
        return self

    def __exit__(self, *a):
        return False


def _timed(name, nbytes=0, flops=0, cycles=0):
    return _TIMER.record(name, nbytes, flops, cycles) if _TIMER is not None else _NoTimer()


def _c(t, dtype=F32):
    return t.contiguous() if t.dtype == dtype else t.to(dtype).contiguous()


def _c16(t):
    """Contiguous fp32 with a 16-B aligned base (the float4 paths of libskp require it): a view
    at an odd storage offset is copied."""
    t = _c(t)
    return t if t.data_ptr() % 16 == 0 else t.clone()


def _rows16(t):
    """fp32 with unit-stride, 16-B aligned rows (row stride a multiple of 4 floats, e.g. a column
    block of a fused projection's output) as it is; anything else through _c16."""
    if (t.dtype == F32 and t.stride(-1) == 1 and t.stride(-2) % 4 == 0 and t.data_ptr() % 16 == 0
            and (t.dim() < 3 or t.shape[0] == 1 or t.stride(0) % 4 == 0)):
        return t
    return _c16(t)


# --------------------------------------------------------------------------- Q·Kᵀ on MFMA
def bgemm(a, b, alpha=1.0, out=None, accumulate=False):
    """out[z] = alpha · a[z] @ b[z] for 3-D fp32 tensors of any strides (skp_bgemm_f32)."""
    _lib.require_device(a, b)
    Z, M, K = a.shape
    Z2, K2, N = b.shape
    assert Z == Z2 and K == K2, (a.shape, b.shape)
    if out is None:
        out = torch.empty(Z, M, N, device=a.device, dtype=F32)
    call("skp_bgemm_f32", ptr(a), a.stride(0), a.stride(1), a.stride(2), ptr(b), b.stride(0), b.stride(1),
         b.stride(2), ptr(out), out.stride(0), out.stride(1), out.stride(2), Z, M, N, K, float(alpha),
         int(accumulate), stream(a.device))
    return out


def bgemm_2b(a, sa, b, sb, out, so, batch, hb, M, N, K, alpha=1.0, accumulate=False):
    """skp_bgemm_f32_2b: for z = o·hb + i, out_z = alpha · a_z @ b_z with operand X_z at
    X + o·sX[0] + i·sX[1], row / column strides sX[2], sX[3] (elements; a: (M, K), b: (K, N),
    out: (M, N))."""
    call("skp_bgemm_f32_2b", ptr(a), *sa, ptr(b), *sb, ptr(out), *so, int(batch), int(hb), int(M), int(N), int(K),
         float(alpha), int(accumulate), stream(a.device))
    return out


class CaptureLogitsHeads(torch.autograd.Function):
    """z = q kᵀ · scale for the B·H heads of a captured layer read in place: q the layer's (B, S, H·d)
    to_q projection, k the ONE (1, N, H·d) to_k projection of the token embedding the batch shares
    (ptp_utils.py:493 / 534) — no head-permute copy of q and no batch-expanded copy of k.  Output
    (B·H, S, N), the head-major layout the capture consumes.  Backward: dq straight into the (B, S,
    H·d) layout; dk per image into a (B, N, H·d) scratch summed over the images (the expand's
    reduction)."""

    @staticmethod
    def forward(ctx, qf, k1, H, scale):
        qf, k1 = _c16(qf), _rows16(k1)
        B, S, C = qf.shape
        N, d, rk = k1.shape[1], C // H, k1.stride(1)
        z = torch.empty(B * H, S, N, device=qf.device, dtype=F32)
        bgemm_2b(qf, (S * C, d, C, 1), k1, (0, d, 1, rk), z, (H * S * N, S * N, N, 1), B * H, H, S, N, d, scale)
        ctx.save_for_backward(qf, k1)
        ctx.meta = (H, float(scale))
        return z

    @staticmethod
    def backward(ctx, dz):
        qf, k1 = ctx.saved_tensors
        H, scale = ctx.meta
        B, S, C = qf.shape
        N, d, rk = k1.shape[1], C // H, k1.stride(1)
        dz = _c16(dz)
        dq = dk1 = None
        if ctx.needs_input_grad[0]:
            dq = torch.empty_like(qf)
            bgemm_2b(dz, (H * S * N, S * N, N, 1), k1, (0, d, rk, 1), dq, (S * C, d, C, 1), B * H, H, S, d, N, scale)
        if ctx.needs_input_grad[1]:
            dkb = torch.empty(B, N, C, device=qf.device, dtype=F32)
            bgemm_2b(dz, (H * S * N, S * N, 1, N), qf, (S * C, d, C, 1), dkb, (N * C, d, C, 1), B * H, H, N, d, S,
                     scale)
            dk1 = dkb.sum(dim=0, keepdim=True) if B > 1 else dkb
        return dq, dk1, None, None


class AttnPVHeads(torch.autograd.Function):
    """out = P v per head into the (B, S, H·d) layout to_out reads: P (B·H, S, N) the captured layer's
    softmax, v the ONE (1, N, H·d) to_v projection of the shared token embedding (ptp_utils.py:
    500-502 / 540-541, the normal-path output of a captured layer) — no batch-expanded copy of v and
    no heads-to-batch permute of the output.  Backward: dP = dout vᵀ; dv per image summed over the
    images."""

    @staticmethod
    def forward(ctx, P, v1, H):
        P, v1 = _c16(P), _rows16(v1)
        BH, S, N = P.shape
        B, C = BH // H, v1.shape[2]
        d, rv = C // H, v1.stride(1)
        out = torch.empty(B, S, C, device=P.device, dtype=F32)
        bgemm_2b(P, (H * S * N, S * N, N, 1), v1, (0, d, rv, 1), out, (S * C, d, C, 1), BH, H, S, d, N)
        ctx.save_for_backward(P, v1)
        ctx.H = H
        return out

    @staticmethod
    def backward(ctx, dout):
        P, v1 = ctx.saved_tensors
        H = ctx.H
        BH, S, N = P.shape
        B, C = BH // H, v1.shape[2]
        d, rv = C // H, v1.stride(1)
        dout = _c16(dout)
        dP = dv1 = None
        if ctx.needs_input_grad[0]:
            dP = torch.empty_like(P)
            bgemm_2b(dout, (S * C, d, C, 1), v1, (0, d, 1, rv), dP, (H * S * N, S * N, N, 1), BH, H, S, N, d)
        if ctx.needs_input_grad[1]:
            dvb = torch.empty(B, N, C, device=P.device, dtype=F32)
            bgemm_2b(P, (H * S * N, S * N, 1, N), dout, (S * C, d, C, 1), dvb, (N * C, d, C, 1), BH, H, N, d, S)
            dv1 = dvb.sum(dim=0, keepdim=True) if B > 1 else dvb
        return dP, dv1, None


def capture_logits_heads(qf, k1, heads, scale):
    """(B·H, S, N) logits of a captured layer from its (B, S, H·d) query projection and the shared
    (1, N, H·d) key projection (CaptureLogitsHeads)."""
    _lib.require_device(qf, k1)
    return CaptureLogitsHeads.apply(qf, k1, int(heads), float(scale))


def attn_pv_heads(P, v1, heads):
    """(B, S, H·d) = per-head P v with the shared (1, N, H·d) value projection (AttnPVHeads)."""
    _lib.require_device(P, v1)
    return AttnPVHeads.apply(P, v1, int(heads))


def heads_eligible(qf, k1, heads):
    """The in-place head GEMMs take fp32 (B, S, H·d) / (1, N, H·d) projections with d, S·H·d and N
    multiples of 4 (16-B aligned heads for the vector loads)."""
    C = qf.shape[-1]
    return (qf.dtype == F32 and k1.dtype == F32 and qf.dim() == 3 and k1.dim() == 3 and k1.shape[0] == 1
            and C % heads == 0 and (C // heads) % 4 == 0 and k1.shape[1] % 4 == 0 and k1.shape[2] == C)


class CaptureLogits(torch.autograd.Function):
    """z = q kᵀ · scale — the layer's cross-attention logits (ptp_utils.py:493 / 534)."""

    @staticmethod
    def forward(ctx, q, k, scale):
        q, k = _c(q), _c(k)
        ctx.save_for_backward(q, k)
        ctx.scale = scale
        return bgemm(q, k.transpose(1, 2), scale)

    @staticmethod
    def backward(ctx, dz):
        q, k = ctx.saved_tensors
        dz = _c(dz)
        dq = dk = None
        if ctx.needs_input_grad[0]:
            dq = bgemm(dz, k, ctx.scale)
        if ctx.needs_input_grad[1]:
            dk = bgemm(dz.transpose(1, 2), q, ctx.scale)
        return dq, dk, None


def capture_logits(q, k, scale):
    return CaptureLogits.apply(q, k, float(scale))


# --------------------------------------------------------------------------- A1 capture
class CaptureAttn(torch.autograd.Function):
    """attn = softmax_N(bicubic_{s→R}(z_low)) — the captured map (ptp_utils.py:513-536)."""

    @staticmethod
    def forward(ctx, z, s, R):
        z = _c(z)
        BH, S, N = z.shape
        assert S == s * s
        attn = torch.empty(BH, R * R, N, device=z.device, dtype=F32)
        with _timed("skp_capture_fwd", (BH * R * R * N + BH * S * N) * 4):
            call("skp_capture_fwd", ptr(z), BH, s, N, R, ptr(attn), None, stream(z.device))
        ctx.save_for_backward(z)
        ctx.s, ctx.R = s, R
        return attn

    @staticmethod
    def backward(ctx, dattn):
        (z,) = ctx.saved_tensors
        return capture_bwd(z, ctx.s, ctx.R, dattn), None, None


def capture_bwd(z, s, R, dattn, gscale=1.0, group=1, strides=None, stats=None):
    """dz_low for g = gscale·dattn; ``dattn`` (BH, R², N) of any strides, or with ``group``/
    ``strides`` = (sb, sp, sn) a per-group gradient (row b uses group b // group).  ``stats``:
    the forward's per-pixel softmax (max, 1/Σ), (BH, R², 2), or None (recomputed)."""
    BH, S, N = z.shape
    if dattn.dtype != F32:
        dattn = dattn.float()
    if strides is None:
        sb, sp, sn = dattn.stride()
        if dattn.shape[0] == 1 and BH > 1:
            sb = 0
    else:
        sb, sp, sn = strides
    ws = torch.empty(BH, R, s, N, device=z.device, dtype=F32)
    dz = torch.empty_like(z)
    with _timed("skp_capture_bwd", (BH * S * N * 2 + BH * R * s * N * 2) * 4):
        call("skp_capture_bwd", ptr(z), BH, s, N, R, ptr(dattn), int(group), sb, sp, sn, float(gscale),
             ptr(stats) if stats is not None else None, ptr(dz), ptr(ws), stream(z.device))
    return dz


def capture_attn(z, s, R):
    return CaptureAttn.apply(z, int(s), int(R))


# --------------------------------------------------------------------------- A3 aggregate
class _Aggregate(torch.autograd.Function):
    @staticmethod
    def forward(ctx, indices, upsample_res, *layers):
        layers = [_c(t) for t in layers]
        BH, RR, N = layers[0].shape
        R = int(round(RR ** 0.5))
        for t in layers:
            if t.shape != layers[0].shape:
                raise ValueError("collect_maps: captured layers must share (BH, R*R, N); got "
                                 f"{[tuple(x.shape) for x in layers]}")
        arr = (ctypes.c_void_p * len(layers))(*[t.data_ptr() for t in layers])
        n_out = N if indices is None else int(indices.numel())
        out = torch.empty(n_out, R, R, device=layers[0].device, dtype=F32)
        idx = None if indices is None else indices.to(device=out.device, dtype=torch.int64).contiguous()
        with _timed("skp_aggregate", (len(layers) * BH * RR * N + n_out * RR) * 4):
            call("skp_aggregate", ctypes.cast(arr, ctypes.POINTER(ctypes.c_void_p)), len(layers), BH, RR, N,
                 ptr(idx), n_out, ptr(out), stream(out.device))
        ctx.meta = (BH, RR, N, R, len(layers))
        ctx.idx = idx
        ctx.upsample_res = upsample_res
        if upsample_res != -1 and upsample_res != R:
            up = torch.empty(n_out, upsample_res, upsample_res, device=out.device, dtype=F32)
            call("skp_resize_bilinear", ptr(out), n_out, R, upsample_res, ptr(up), stream(out.device))
            out = up
        return out

    @staticmethod
    def backward(ctx, dmap):
        BH, RR, N, R, L = ctx.meta
        dmap = _c(dmap)
        if ctx.upsample_res != -1 and ctx.upsample_res != R:
            g = torch.empty(dmap.shape[0], R, R, device=dmap.device, dtype=F32)
            call("skp_resize_bilinear_bwd", ptr(dmap), dmap.shape[0], R, ctx.upsample_res, ptr(g), stream(dmap.device))
            dmap = g
        dmap = dmap.reshape(-1, RR) / float(L * BH)
        if ctx.idx is not None:
            full = torch.zeros(N, RR, device=dmap.device, dtype=F32)
            full.index_add_(0, ctx.idx, dmap)
            dmap = full
        # d attn_l[b, p, n] = dmap[n, p] / (L·BH): a stride-0 broadcast view, never materialised
        g = dmap.t().unsqueeze(0).expand(BH, RR, N)
        return (None, None) + tuple(g for _ in range(L))


def aggregate(layers, indices=None, upsample_res=-1):
    return _Aggregate.apply(indices, int(upsample_res), *layers)


FUSED_MAPS = True   # tests switch it: False = skp_capture_fwd + skp_aggregate (the AttentionStore path)


def capture_maps_bytes(B, H, N, R, sizes):
    """Algorithmic HBM bytes of one skp_capture_maps_fwd launch: every z_low read once, the
    (B, N, R²) maps and the (B·H, R², 2) per-layer stats written once."""
    RR = R * R
    return 4 * (sum(B * H * s * s * N for s in sizes) + B * N * RR + len(sizes) * B * H * RR * 2)


def capture_maps_flops(B, H, N, R, sizes):
    """Algorithmic fp32 VALU work of one skp_capture_maps_fwd launch: per
    (image, head, layer, pixel, token) 15 FLOP — horizontal bicubic 4 multiply-adds (8), softmax
    max 1 + (z − m)·log2e as an FMA 2 + exp 1 + Σ 1, normalise-and-accumulate FMA 2 — and per
    (image, head, layer, output row, low-res column, token) 8 for the vertical bicubic pass."""
    return sum(B * H * N * (15 * R * R + 8 * R * s) for s in sizes)


# VALU issue cost on gfx950 (MI355X_MICROARCH.md, "vector-instruction ISSUE cost"): a wave64
# instruction occupies its SIMD 4 cycles (v_fma_f32 / v_pk_fma_f32 / v_max3_f32 …), 8 for the
# transcendentals (v_exp_f32); a packed f32 instruction does 2 elements per lane.  SIMD-cycles per
# element of one f32 op: packed 4/128, transcendental 8/64.
_PK, _TR = 4.0 / 128, 8.0 / 64


def capture_maps_issue_cycles(B, H, N, R, sizes):
    """Minimal VALU issue cycles (summed over SIMDs) of one skp_capture_maps_fwd launch: per (image,
    head, layer, pixel, token) the 4 horizontal taps (4 packed FMA), the max (½ v_max3), the exp
    argument (1 packed FMA), v_exp_f32 (transcendental), Σ (1 packed add) and the normalised
    accumulate (1 packed FMA); per (row, low-res column, token) the 4 vertical taps."""
    per_px = 4 * _PK + 0.5 * 4.0 / 64 + _PK + _TR + _PK + _PK
    return sum(B * H * N * (per_px * R * R + 4 * _PK * R * s) for s in sizes)


def capture_maps_sel_bwd_issue_cycles(B, H, N, R, sizes):
    """Minimal VALU issue cycles of the dense part of skp_capture_maps_bwd_sel: per (image, head,
    layer, pixel, token) 4 horizontal taps, the exp argument, v_exp_f32, ×(−dot) and the 4-tap
    horizontal adjoint (packed f32 except the exp); per (row, low-res column, token) the vertical
    pass and the vertical adjoint (4 + 4 packed FMA)."""
    per_px = 4 * _PK + _PK + _TR + _PK + 4 * _PK
    return sum(B * H * N * (per_px * R * R + 8 * _PK * R * s) for s in sizes)


def capture_maps_bwd_flops(B, H, N, R, sizes):
    """Algorithmic fp32 VALU work of one skp_capture_maps_bwd call: per (image, head, layer,
    pixel, token) 24 FLOP — rebuild the softmax row (taps 8, exp argument 2, exp 1, ×1/Σ 1), a·g 1,
    Σ a·g 1, dZ = a·g − a·dot 2, horizontal adjoint 4 multiply-adds (8) — and per (row, low-res
    column, token) 8 each for the vertical pass and the vertical adjoint."""
    return sum(B * H * N * (24 * R * R + 16 * R * s) for s in sizes)


def capture_maps_bwd_bytes(B, H, N, R, sizes):
    """Algorithmic HBM bytes of one skp_capture_maps_bwd call: the map gradient read once (and
    its pixel-major copy written and read once), every z_low and stats read once, the row
    partials written and read once, dz_low written once."""
    RR = R * R
    return 4 * (3 * B * N * RR + sum(2 * B * H * s * s * N + 2 * B * H * RR + 2 * B * H * R * s * N for s in sizes))


class CaptureMaps(torch.autograd.Function):
    """Per-image maps straight from the captured layers' logits (fused capture + aggregate).

    zs[l]: (B·H, s_l², N) logits of captured layer l.  Output (B, N, R, R):
    map[b] = mean over layers and the H heads of image b of softmax(bicubic(z)).
    One launch of skp_capture_maps_fwd: the (B·H, R², N) attention is never written; only the
    per-pixel softmax stats are kept for the backward, which hands each layer's kernel the
    per-image map gradient as a broadcast (group = H), so no (B·H, R², N) gradient is
    materialised either.
    """

    @staticmethod
    def forward(ctx, B, R, sizes, *zs):
        zs = [_c16(z) for z in zs]
        BH, _, N = zs[0].shape
        H = BH // B
        L = len(zs)
        dev = zs[0].device
        RR = R * R
        if FUSED_MAPS:
            out, stats = _capture_maps_run(zs, sizes, B, R)
        else:
            # per-pixel softmax (max, 1/Σ) of every layer, kept for the backward (8 B per pixel-head)
            stats = [torch.empty(BH, RR, 2, device=dev, dtype=F32) for _ in range(L)]
            out = torch.empty(B, N, R, R, device=dev, dtype=F32)
            attn = [torch.empty(BH, RR, N, device=dev, dtype=F32) for _ in range(L)]
            for z, a, st, s in zip(zs, attn, stats, sizes):
                with _timed("skp_capture_fwd", (BH * RR * N + BH * s * s * N) * 4):
                    call("skp_capture_fwd", ptr(z), BH, s, N, R, ptr(a), ptr(st), stream(dev))
            for b in range(B):
                off = b * H * RR * N * 4
                arr = (ctypes.c_void_p * L)(*[a.data_ptr() + off for a in attn])
                with _timed("skp_aggregate", (L * H * RR * N + N * RR) * 4):
                    call("skp_aggregate", ctypes.cast(arr, ctypes.POINTER(ctypes.c_void_p)), L, H, RR, N, None, N,
                         ptr(out[b]), stream(dev))
            del attn
        ctx.save_for_backward(*zs, *stats)
        ctx.meta = (B, H, R, N, list(sizes))
        return out

    @staticmethod
    def backward(ctx, dmaps):
        saved = ctx.saved_tensors
        L = len(saved) // 2
        return (None, None, None) + tuple(CaptureMaps._dense_bwd(saved[:L], saved[L:], ctx.meta, dmaps))

    @staticmethod
    def _dense_bwd(zs, stats, meta, dmaps):
        """dz_low of every layer for a dense per-image map gradient dmaps (B, N, R, R)."""
        B, H, R, N, sizes = meta
        dmaps = _c(dmaps)                       # (B, N, R, R)
        RR = R * R
        scale = 1.0 / float(len(zs) * H)
        L = len(zs)
        if FUSED_MAPS and N % 4 == 0:
            dzs = [torch.empty_like(z) for z in zs]
            ws = torch.empty(B * RR * N + B * H * R * max(sizes) * N, device=dmaps.device, dtype=F32)
            zp = (ctypes.c_void_p * L)(*[z.data_ptr() for z in zs])
            sp = (ctypes.c_int * L)(*[int(s) for s in sizes])
            stp = (ctypes.c_void_p * L)(*[st.data_ptr() for st in stats])
            dp = (ctypes.c_void_p * L)(*[d.data_ptr() for d in dzs])
            with _timed("skp_capture_maps_bwd", capture_maps_bwd_bytes(B, H, N, R, sizes),
                        capture_maps_bwd_flops(B, H, N, R, sizes)):
                call("skp_capture_maps_bwd", ctypes.cast(zp, ctypes.POINTER(ctypes.c_void_p)), sp, L, B, H, N, R,
                     ptr(dmaps), scale, ctypes.cast(stp, ctypes.POINTER(ctypes.c_void_p)),
                     ctypes.cast(dp, ctypes.POINTER(ctypes.c_void_p)), ptr(ws), stream(dmaps.device))
            del ws
        else:
            dzs = [capture_bwd(z, s, R, dmaps, gscale=scale, group=H, strides=(N * RR, 1, RR), stats=st)
                   for z, s, st in zip(zs, sizes, stats)]
        return dzs


def capture_maps(zs, sizes, B, R):
    """Per-image (B, N, R, R) maps from captured logits (see CaptureMaps)."""
    return CaptureMaps.apply(int(B), int(R), tuple(int(s) for s in sizes), *zs)


# A/B: 0 = the selected rows' gradient goes through the dense (B, N, R²) map gradient and
# skp_capture_maps_bwd, as in r02
SEL_BWD = True   # tests switch it: False = the dense map gradient + skp_capture_maps_bwd
# skp_capture_maps_bwd_sel's per-image row limit (32-bit lane masks in csrc/skp_capture_sel.hip);
# more selected rows per image (a user --top_k > 32) take the dense backward
SEL_MAXK = 32


def capture_maps_sel_bwd_bytes(B, H, N, R, sizes, K):
    """Algorithmic HBM bytes of one skp_capture_maps_bwd_sel call (fast path), per layer: z_low read
    and dz_low written once, the stats read once, the per-pixel (mb, d) pairs and the K selected
    rows' e = a·g written and read once, the K gradient rows read once."""
    RR = R * R
    BH = B * H
    return 4 * sum(2 * BH * s * s * N + 2 * BH * RR + 4 * BH * RR + 2 * BH * K * RR + B * K * RR for s in sizes)


def capture_maps_sel_bwd_flops(B, H, N, R, sizes):
    """Algorithmic fp32 VALU work of the dense part of skp_capture_maps_bwd_sel: per (image, head,
    layer, pixel, token) 20 FLOP — rebuild a (taps 8, exp argument 2, exp 1), ×(−dot) 1, horizontal
    adjoint 8 — and per (row, low-res column, token) 8 each for the vertical pass and the vertical
    adjoint.  (The sparse part, K tokens per pixel, is not counted.)"""
    return sum(B * H * N * (20 * R * R + 16 * R * s) for s in sizes)


class CapturedMaps:
    """The fused capture's per-image maps (B, N, R, R) — computed without an autograd graph —
    plus what the backward needs (the logits ``zs`` with their graph, the per-pixel softmax stats).

    ``maps`` feeds the selection (no gradient, as in the reference: top-k / FPS run on detached
    maps); ``select(rows)`` gathers the selected token rows of every image as ONE differentiable
    (M, R, R) tensor whose backward is the sparse ``skp_capture_maps_bwd_sel``: the K selected rows'
    gradient goes straight to the kernel, and no (B, N, R²) map gradient is ever formed
    (reference optimize.py:403-424 only differentiates maps[top_embedding_indices])."""

    def __init__(self, zs, sizes, B, R):
        self.zs = list(zs)
        # called once by select()'s backward right after the capture backward is enqueued (on the
        # autograd thread, the main stream current), then cleared
        self.after_backward = None
        self.sizes = tuple(int(s) for s in sizes)
        self.B, self.R = int(B), int(R)
        with torch.no_grad():
            self.maps, self.stats = _capture_maps_run([z.detach() for z in self.zs], self.sizes, self.B, self.R)
        BH, _, N = self.zs[0].shape
        self.H, self.N = BH // self.B, N

    def select(self, rows):
        """rows: per image a 1-D int64 tensor of token ids (or None) -> cat_b maps[b, rows[b]]."""
        if len(rows) != self.B:
            raise ValueError(f"select: {len(rows)} row lists for {self.B} images")
        counts = [0 if r is None else int(r.numel()) for r in rows]
        toks = [r.to(device=self.maps.device, dtype=torch.int64).reshape(-1) for r, c in zip(rows, counts) if c]
        tok = torch.cat(toks) if toks else torch.empty(0, dtype=torch.int64, device=self.maps.device)
        return _SelectMaps.apply(self, tok, tuple(counts), *self.zs)


def _capture_maps_run(zs, sizes, B, R):
    """skp_capture_maps_fwd: (maps (B, N, R, R), per-layer stats (B·H, R², 2))."""
    zs = [_c16(z) for z in zs]
    BH, _, N = zs[0].shape
    H = BH // B
    L = len(zs)
    dev = zs[0].device
    RR = R * R
    stats = [torch.empty(BH, RR, 2, device=dev, dtype=F32) for _ in range(L)]
    out = torch.empty(B, N, R, R, device=dev, dtype=F32)
    zp = (ctypes.c_void_p * L)(*[z.data_ptr() for z in zs])
    sp = (ctypes.c_int * L)(*[int(s) for s in sizes])
    stp = (ctypes.c_void_p * L)(*[st.data_ptr() for st in stats])
    with _timed("skp_capture_maps_fwd", capture_maps_bytes(B, H, N, R, sizes), capture_maps_flops(B, H, N, R, sizes),
                capture_maps_issue_cycles(B, H, N, R, sizes)):
        call("skp_capture_maps_fwd", ctypes.cast(zp, ctypes.POINTER(ctypes.c_void_p)), sp, L, B, H, N, R,
             ptr(out), ctypes.cast(stp, ctypes.POINTER(ctypes.c_void_p)), stream(dev))
    return out, stats


def capture_maps_bwd_sel(zs, sizes, B, R, tok_table, gsel, gscale, stats):
    """dz_low of every layer for a sparse per-image map gradient: image b's gradient is
    gsel[b, k] (R²) at token tok_table[b, k] (−1 = unused), zero elsewhere (skp_capture_maps_bwd_sel)."""
    zs = [_c16(z) for z in zs]
    BH, _, N = zs[0].shape
    H = BH // B
    L = len(zs)
    K = tok_table.shape[1]
    dev = zs[0].device
    sp = (ctypes.c_int * L)(*[int(s) for s in sizes])
    nws = _lib.lib().skp_capture_maps_bwd_sel_workspace(sp, L, B, H, N, R, K)
    if nws < 0:
        raise ValueError(f"capture_maps_bwd_sel: bad shape B={B} H={H} N={N} R={R} K={K} sizes={sizes}")
    ws = torch.empty(int(nws), device=dev, dtype=F32)
    dzs = [torch.empty_like(z) for z in zs]
    arr = lambda ts: ctypes.cast((ctypes.c_void_p * L)(*[t.data_ptr() for t in ts]),   # noqa: E731
                                 ctypes.POINTER(ctypes.c_void_p))
    tok_table = tok_table.to(device=dev, dtype=torch.int64).contiguous()
    gsel = _c(gsel)
    with _timed("skp_capture_maps_bwd_sel", capture_maps_sel_bwd_bytes(B, H, N, R, sizes, K),
                capture_maps_sel_bwd_flops(B, H, N, R, sizes), capture_maps_sel_bwd_issue_cycles(B, H, N, R, sizes)):
        call("skp_capture_maps_bwd_sel", arr(zs), sp, L, B, H, N, R, ptr(tok_table), K, ptr(gsel), float(gscale),
             arr(stats), arr(dzs), ptr(ws), stream(dev))
    return dzs


class _SelectMaps(torch.autograd.Function):
    """cat_b maps[b, rows_b] with the sparse capture backward (see CapturedMaps.select)."""

    @staticmethod
    def forward(ctx, cm, tok, counts, *zs):
        B, N, R = cm.B, cm.N, cm.R
        img = torch.cat([torch.full((c,), b, dtype=torch.int64, device=tok.device) for b, c in enumerate(counts) if c]) \
            if tok.numel() else tok
        out = cm.maps.view(B * N, R * R)[img * N + tok].view(-1, R, R)
        ctx.cm, ctx.counts = cm, counts
        ctx.save_for_backward(tok)
        return out

    @staticmethod
    def backward(ctx, g):
        cm, counts = ctx.cm, ctx.counts
        (tok,) = ctx.saved_tensors
        B, N, R, L = cm.B, cm.N, cm.R, len(cm.zs)
        RR = R * R
        K = max(max(counts), 1)
        g = _c(g).view(-1, RR)
        scale = 1.0 / float(L * cm.H)
        if SEL_BWD and N % 4 == 0 and K <= SEL_MAXK:
            # (B, K) token table (−1 pads) and the (B, K, R²) gradient rows, in row order per image
            tt = torch.full((B, K), -1, dtype=torch.int64, device=g.device)
            gs = torch.zeros(B, K, RR, dtype=F32, device=g.device)
            off = 0
            for b, c in enumerate(counts):
                if c:
                    tt[b, :c] = tok[off:off + c]
                    gs[b, :c] = g[off:off + c]
                    off += c
            dzs = capture_maps_bwd_sel(cm.zs, cm.sizes, B, R, tt, gs, scale, cm.stats)
        else:
            dense = torch.zeros(B * N, RR, dtype=F32, device=g.device)
            img = torch.cat([torch.full((c,), b, dtype=torch.int64, device=g.device) for b, c in enumerate(counts) if c])
            dense.index_add_(0, img * N + tok, g)
            dzs = CaptureMaps._dense_bwd([_c(z) for z in cm.zs], cm.stats, (B, cm.H, R, N, list(cm.sizes)),
                                         dense.view(B, N, R, R))
        cb, cm.after_backward = cm.after_backward, None
        if cb is not None:    # e.g. TokenOptimizer's VAE prefetch, enqueued behind the capture backward
            cb()
        return (None, None, None) + tuple(dzs)


class _Resize(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, Ro):
        x = _c(x)
        C, R, _ = x.shape
        out = torch.empty(C, Ro, Ro, device=x.device, dtype=F32)
        call("skp_resize_bilinear", ptr(x), C, R, Ro, ptr(out), stream(x.device))
        ctx.R = R
        return out

    @staticmethod
    def backward(ctx, g):
        g = _c(g)
        C, Ro, _ = g.shape
        gin = torch.empty(C, ctx.R, ctx.R, device=g.device, dtype=F32)
        call("skp_resize_bilinear_bwd", ptr(g), C, ctx.R, Ro, ptr(gin), stream(g.device))
        return gin, None


def resize_bilinear(x, Ro):
    """(C, R, R) -> (C, Ro, Ro), F.interpolate(bilinear, align_corners=False) (optimize.py:63-70)."""
    _lib.require_device(x)
    return _Resize.apply(x, int(Ro))


# --------------------------------------------------------------------------- A4-A6 argmax family
def find_max_pixel(maps):
    _lib.require_device(maps)
    maps = _c(maps)
    T, h, w = maps.shape
    pos = torch.empty(T, 2, device=maps.device, dtype=F32)
    call("skp_argmax2d", ptr(maps), T, h, w, None, 0, ptr(pos), None, stream(maps.device))
    return pos


def argmax_index(maps):
    maps = _c(maps)
    T, h, w = maps.shape
    idx = torch.empty(T, device=maps.device, dtype=torch.int64)
    call("skp_argmax2d", ptr(maps), T, h, w, None, 0, None, ptr(idx), stream(maps.device))
    return idx


def _radius2(h):
    r = 0.05 * h
    return float(r ** 2)


def find_k_max_pixels(maps, num=3, return_masked=False):
    _lib.require_device(maps)
    maps = _c(maps)
    T, h, w = maps.shape
    pos = torch.empty(num, T, 2, device=maps.device, dtype=F32)
    masked = torch.empty_like(maps) if return_masked else None
    call("skp_k_max_pixels", ptr(maps), T, h, w, int(num), _radius2(h), ptr(pos), ptr(masked), stream(maps.device))
    return (pos, masked) if return_masked else pos


def mask_radius(maps, max_coords, radius):
    _lib.require_device(maps)
    maps = _c(maps)
    T, h, w = maps.shape
    out = torch.empty_like(maps)
    call("skp_mask_radius", ptr(maps), T, h, w, ptr(_c(max_coords)), float(radius) ** 2, ptr(out),
         stream(maps.device))
    return out


def pixel_from_weighted_avg(heatmaps, distance=5):
    """Mutates ``heatmaps`` in place like the reference (eval.py:137) when it is contiguous fp32."""
    _lib.require_device(heatmaps)
    T, h, w = heatmaps.shape
    work = heatmaps if (heatmaps.is_contiguous() and heatmaps.dtype == F32) else heatmaps.float().contiguous()
    pos = torch.empty(T, 2, device=heatmaps.device, dtype=F32)
    call("skp_weighted_avg", ptr(work), T, h, w, float(distance) if distance != -1 else -1.0, 1, ptr(pos),
         stream(heatmaps.device))
    if work is not heatmaps:
        heatmaps.copy_(work)
    return pos


# --------------------------------------------------------------------------- A7 targets
def gaussian_circles(pos, size, sigma):
    """pos (num, T, 2) in [0,1] -> (T, size, size); (T, 2) is treated as num = 1."""
    _lib.require_device(pos)
    pos = _c(pos)
    if pos.dim() == 2:
        pos = pos.unsqueeze(0)
    num, T, _ = pos.shape
    out = torch.empty(T, size, size, device=pos.device, dtype=F32)
    call("skp_gaussian_target", ptr(pos), num, T, int(size), float(sigma), ptr(out), stream(pos.device))
    return out


# --------------------------------------------------------------------------- A8-A10 selection
def find_top_k_gaussian(maps, top_k, sigma=3, epsilon=1e-5, num_subjects=1, return_kl=False):
    _lib.require_device(maps)
    maps = _c(maps)
    T, h, w = maps.shape
    top_k = min(int(top_k), T)   # argsort(kl)[:top_k] (ptp_utils.py:110): at most T candidates
    out = torch.empty(top_k, device=maps.device, dtype=torch.int64)
    kl = torch.empty(T, device=maps.device, dtype=torch.float64)
    call("skp_topk_gaussian", ptr(maps), T, h, w, int(top_k), float(sigma), float(epsilon), int(num_subjects),
         ptr(out), ptr(kl), ptr(kl), stream(maps.device))
    return (out, kl) if return_kl else out


# the A8 top-k as its own ranking launch behind the KL kernel (the fused one-launch form measured
# 2.5× slower, profiles/r05w_a8_fused_ab.txt, and was removed in r06)
def find_top_k_gaussian_batch(maps, top_k, sigma=3, epsilon=1e-5, num_subjects=1):
    """find_top_k_gaussian of every image of a (nb, T, h, w) stack in one launch each for the KL
    ranking and the sort: (nb, top_k) int64, row b = find_top_k_gaussian(maps[b], ...)."""
    _lib.require_device(maps)
    maps = _c(maps)
    nb, T, h, w = maps.shape
    top_k = min(int(top_k), T)
    out = torch.empty(nb, top_k, device=maps.device, dtype=torch.int64)
    kl = torch.empty(nb, T, device=maps.device, dtype=torch.float64)
    # the whole A8 call (algorithmic bytes: every map read once, the keys written) in one timed
    # scope: the KL ranking launch and the ranking of the keys
    with _timed("skp_topk_gaussian_batch", maps.numel() * 4 + nb * T * 8):
        # the KL ranking launch, then (top_k > 0) the ranking of its keys, both on this stream
        call("skp_topk_gaussian_batch", ptr(maps), nb, T, h, w, int(top_k), float(sigma), float(epsilon),
             int(num_subjects), ptr(out), ptr(kl), ptr(kl), stream(maps.device))
    return out


def furthest_point_sampling_batch(maps, top_k, candidates):
    """furthest_point_sampling of every image of a (nb, T, h, w) stack, candidates (nb, C) token
    ids per image, in one argmax and one FPS launch.  Returns ((nb, top_k) int64, (nb,) int32)."""
    _lib.require_device(maps)
    maps = _c(maps)
    nb, T, h, w = maps.shape
    cand = candidates.to(device=maps.device, dtype=torch.int64).contiguous()
    if cand.dim() != 2 or cand.shape[0] != nb:
        raise ValueError(f"candidates {tuple(cand.shape)} for {nb} images")
    out = torch.empty(nb, top_k, device=maps.device, dtype=torch.int64)
    n_out = torch.empty(nb, device=maps.device, dtype=torch.int32)
    ws = torch.empty(2 * cand.numel() + 2, device=maps.device, dtype=F32)
    call("skp_fps_batch", ptr(maps), nb, T, h, w, ptr(cand), cand.shape[1], int(top_k), ptr(out), ptr(n_out),
         ptr(ws), stream(maps.device))
    return out, n_out


def fps_from_keys_batch(keys, maps, n_cand, top_k):
    """Per image b: the n_cand tokens of smallest keys[b] (torch.argsort order: NaN last, ties by
    index), then furthest_point_sampling(maps[b], top_k, those candidates) — skp_fps_keys_batch:
    the ranking and the candidates' argmax in one launch, then FPS.  keys (nb, T) float64, maps
    (nb, T, h, w).  Returns ((nb, top_k) int64, (nb,) int32 counts, (nb, n_cand) candidates)."""
    _lib.require_device(maps)
    maps = _c(maps)
    nb, T, h, w = maps.shape
    keys = keys.to(device=maps.device, dtype=torch.float64).contiguous()
    if tuple(keys.shape) != (nb, T):
        raise ValueError(f"keys {tuple(keys.shape)} for maps {tuple(maps.shape)}")
    n_cand = min(int(n_cand), T)
    dev = maps.device
    cand = torch.empty(nb, n_cand, device=dev, dtype=torch.int64)
    out = torch.empty(nb, top_k, device=dev, dtype=torch.int64)
    n_out = torch.empty(nb, device=dev, dtype=torch.int32)
    ws = torch.empty(2 * nb * n_cand + 2, device=dev, dtype=F32)
    call("skp_fps_keys_batch", ptr(keys), ptr(maps), nb, T, h, w, n_cand, int(top_k), ptr(cand), ptr(out), ptr(n_out),
         ptr(ws), stream(dev))
    return out, n_out, cand


def gaussian_fps_batch(maps, maps_t, n_cand, top_k, sigma=3, epsilon=1e-5, num_subjects=1):
    """The training pass's selection for every image of a stack (optimize.py:403-410 per replica):
    candidates = find_top_k_gaussian(maps[b], n_cand), then
    furthest_point_sampling(maps_t[b], top_k, candidates) — maps (nb, T, h, w) the images' maps,
    maps_t the maps the FPS reads (the warps').  Three launches: the KL keys
    (skp_topk_gaussian_batch, top_k 0), the ranking + the candidates' argmax on maps_t, FPS.
    Returns what fps_from_keys_batch returns: identical to find_top_k_gaussian_batch +
    furthest_point_sampling_batch."""
    _lib.require_device(maps)
    maps = _c(maps)
    nb, T, h, w = maps.shape
    if tuple(maps_t.shape) != (nb, T, h, w):
        raise ValueError(f"maps_t {tuple(maps_t.shape)} for maps {tuple(maps.shape)}")
    kl = torch.empty(nb, T, device=maps.device, dtype=torch.float64)
    # one timed scope for the pass's whole selection chain (bench: `selection`)
    with _timed("skp_selection", maps.numel() * 4 + nb * T * 8 + nb * min(int(n_cand), T) * h * w * 4):
        with _timed("skp_topk_gaussian_batch", maps.numel() * 4 + nb * T * 8):
            call("skp_topk_gaussian_batch", ptr(maps), nb, T, h, w, 0, float(sigma), float(epsilon),
                 int(num_subjects), ptr(kl), ptr(kl), ptr(kl), stream(maps.device))
        return fps_from_keys_batch(kl, maps_t, n_cand, top_k)


def entropy_keys_batch(maps):
    """The softmax entropies of every row of a (nb, T, h, w) stack (ptp_utils.py:179-182) in one
    launch: (nb, T) float64, the keys entropy_sort ranks ascending."""
    _lib.require_device(maps)
    maps = _c(maps)
    nb, T, h, w = maps.shape
    ent = torch.empty(nb, T, device=maps.device, dtype=torch.float64)
    call("skp_entropy_sort", ptr(maps), nb * T, h, w, 0, ptr(ent), ptr(ent), ptr(ent), stream(maps.device))
    return ent


def entropy_sort_batch(maps, top_k):
    """entropy_sort of every image of a (nb, T, h, w) stack: the entropies of all nb·T rows in one
    launch (skp_entropy_sort's kernel, no ranking), then the per-image ascending top_k of them in
    one skp_topk_keys launch.  (nb, top_k) int64, row b = entropy_sort(maps[b], top_k)."""
    _lib.require_device(maps)
    maps = _c(maps)
    nb, T, h, w = maps.shape
    top_k = min(int(top_k), T)
    out = torch.empty(nb, top_k, device=maps.device, dtype=torch.int64)
    ent = torch.empty(nb, T, device=maps.device, dtype=torch.float64)
    call("skp_entropy_sort", ptr(maps), nb * T, h, w, 0, ptr(out), ptr(ent), ptr(ent), stream(maps.device))
    if top_k > 0:
        call("skp_topk_keys", ptr(ent), nb, T, int(top_k), ptr(out), stream(maps.device))
    return out


def entropy_sort(maps, top_k, return_entropy=False):
    _lib.require_device(maps)
    maps = _c(maps)
    T, h, w = maps.shape
    top_k = min(int(top_k), T)   # argsort(entropy)[:top_k] (ptp_utils.py:185): at most T candidates
    out = torch.empty(top_k, device=maps.device, dtype=torch.int64)
    ent = torch.empty(T, device=maps.device, dtype=torch.float64)
    call("skp_entropy_sort", ptr(maps), T, h, w, int(top_k), ptr(out), ptr(ent), ptr(ent), stream(maps.device))
    return (out, ent) if return_entropy else out


def furthest_point_sampling(maps, top_k, candidates):
    """Returns (selected int64 (top_k,), count int32 device scalar)."""
    _lib.require_device(maps)
    maps = _c(maps)
    T, h, w = maps.shape
    cand = candidates.to(device=maps.device, dtype=torch.int64).contiguous()
    out = torch.empty(top_k, device=maps.device, dtype=torch.int64)
    n_out = torch.empty(1, device=maps.device, dtype=torch.int32)
    ws = torch.empty(2 * cand.numel() + 2, device=maps.device, dtype=F32)
    call("skp_fps", ptr(maps), T, h, w, ptr(cand), cand.numel(), int(top_k), ptr(out), ptr(n_out), ptr(ws),
         stream(maps.device))
    return out, n_out


# --------------------------------------------------------------------------- A11 / A12 losses
class SharpeningLoss(torch.autograd.Function):
    @staticmethod
    def forward(ctx, A, sigma, num_subjects):
        A = _c(A)
        T, h, w = A.shape
        pos = torch.empty(num_subjects, T, 2, device=A.device, dtype=F32)
        part = torch.empty(T, device=A.device, dtype=torch.float64)
        loss = torch.empty((), device=A.device, dtype=F32)
        call("skp_sharpen_fwd", ptr(A), T, h, w, float(sigma), int(num_subjects), ptr(pos), ptr(part), ptr(loss),
             stream(A.device))
        ctx.save_for_backward(A, pos)
        ctx.sigma, ctx.num = sigma, num_subjects
        return loss

    @staticmethod
    def backward(ctx, g):
        A, pos = ctx.saved_tensors
        T, h, w = A.shape
        dA = torch.empty_like(A)
        call("skp_sharpen_bwd", ptr(A), T, h, w, float(ctx.sigma), int(ctx.num), ptr(pos), ptr(_c(g.reshape(1))),
             ptr(dA), stream(A.device))
        return dA, None, None


def sharpening_loss(A, sigma=1.0, num_subjects=1):
    _lib.require_device(A)
    return SharpeningLoss.apply(A, float(sigma), int(num_subjects))


class SharpeningLossBatch(torch.autograd.Function):
    """SharpeningLoss of nb images' selected rows at once: A (nb·T, h, w) → (nb,) losses, each the
    single-image loss (skp_sharpen_fwd_batch / _bwd_batch: one launch per direction)."""

    @staticmethod
    def forward(ctx, A, nb, sigma, num_subjects):
        A = _c(A)
        R, h, w = A.shape
        T = R // nb
        pos = torch.empty(num_subjects, R, 2, device=A.device, dtype=F32)
        part = torch.empty(R, device=A.device, dtype=torch.float64)
        loss = torch.empty(nb, device=A.device, dtype=F32)
        call("skp_sharpen_fwd_batch", ptr(A), nb, T, h, w, float(sigma), int(num_subjects), ptr(pos), ptr(part),
             ptr(loss), stream(A.device))
        ctx.save_for_backward(A, pos)
        ctx.meta = (nb, T, sigma, num_subjects)
        return loss

    @staticmethod
    def backward(ctx, g):
        A, pos = ctx.saved_tensors
        nb, T, sigma, num = ctx.meta
        _, h, w = A.shape
        dA = torch.empty_like(A)
        call("skp_sharpen_bwd_batch", ptr(A), nb, T, h, w, float(sigma), int(num), ptr(pos), ptr(_c(g.reshape(nb))),
             ptr(dA), stream(A.device))
        return dA, None, None, None


def sharpening_loss_batch(A, nb, sigma=1.0, num_subjects=1):
    """(nb,) sharpening losses of nb images whose T selected rows each are stacked in A (nb·T, h, w)."""
    _lib.require_device(A)
    if A.shape[0] % nb:
        raise ValueError(f"{A.shape[0]} rows for {nb} images")
    return SharpeningLossBatch.apply(A, int(nb), float(sigma), int(num_subjects))


class AffineWarp(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, theta):
        x = _c(x)
        B, C, H, W = x.shape
        th = _c(theta.to(x.device))
        out = torch.empty_like(x)
        call("skp_affine_warp", ptr(x), B, C, H, W, ptr(th), ptr(out), stream(x.device))
        ctx.save_for_backward(th)
        ctx.shape = (B, C, H, W)
        return out

    @staticmethod
    def backward(ctx, g):
        (th,) = ctx.saved_tensors
        B, C, H, W = ctx.shape
        gin = torch.empty(B, C, H, W, device=g.device, dtype=F32)
        call("skp_affine_warp_bwd", ptr(_c(g)), B, C, H, W, ptr(th), ptr(gin), stream(g.device))
        return gin, None


def affine_warp(x, theta):
    """grid_sample(x, affine_grid(theta)) (bilinear, zeros, align_corners=False); x (B,C,H,W)."""
    _lib.require_device(x)
    return AffineWarp.apply(x, theta)


class EquivarianceLoss(torch.autograd.Function):
    @staticmethod
    def forward(ctx, A, At, theta_inv):
        A, At = _c(A), _c(At)
        T, h, w = A.shape
        th = _c(theta_inv.to(A.device)).reshape(6)
        part = torch.empty(T, device=A.device, dtype=torch.float64)
        loss = torch.empty((), device=A.device, dtype=F32)
        call("skp_equiv_fwd", ptr(A), ptr(At), T, h, w, ptr(th), ptr(part), ptr(loss), stream(A.device))
        ctx.save_for_backward(A, At, th)
        return loss

    @staticmethod
    def backward(ctx, g):
        A, At, th = ctx.saved_tensors
        T, h, w = A.shape
        dA = torch.empty_like(A) if ctx.needs_input_grad[0] else None
        dAt = torch.empty_like(At)
        call("skp_equiv_bwd", ptr(A), ptr(At), T, h, w, ptr(th), ptr(_c(g.reshape(1))), ptr(dA), ptr(dAt),
             stream(A.device))
        return dA, (dAt if ctx.needs_input_grad[1] else None), None


def equivariance_loss_single(A, At, theta_inv):
    """mean((A − warp(At, theta_inv))²) with gradients into A and At."""
    _lib.require_device(A, At)
    return EquivarianceLoss.apply(A, At, theta_inv)


class EquivarianceLossBatch(torch.autograd.Function):
    """EquivarianceLoss of nb replicas at once: A, At (nb·T, h, w), theta_inv (nb, 2, 3) → (nb,)
    losses, each the single-replica loss (skp_equiv_fwd_batch / _bwd_batch)."""

    @staticmethod
    def forward(ctx, A, At, theta_inv, nb):
        A, At = _c(A), _c(At)
        R, h, w = A.shape
        T = R // nb
        th = _c(theta_inv.to(A.device)).reshape(nb * 6)
        part = torch.empty(R, device=A.device, dtype=torch.float64)
        loss = torch.empty(nb, device=A.device, dtype=F32)
        call("skp_equiv_fwd_batch", ptr(A), ptr(At), nb, T, h, w, ptr(th), ptr(part), ptr(loss), stream(A.device))
        ctx.save_for_backward(A, At, th)
        ctx.meta = (nb, T)
        return loss

    @staticmethod
    def backward(ctx, g):
        A, At, th = ctx.saved_tensors
        nb, T = ctx.meta
        _, h, w = A.shape
        dA = torch.empty_like(A) if ctx.needs_input_grad[0] else None
        dAt = torch.empty_like(At)
        call("skp_equiv_bwd_batch", ptr(A), ptr(At), nb, T, h, w, ptr(th), ptr(_c(g.reshape(nb))), ptr(dA), ptr(dAt),
             stream(A.device))
        return dA, (dAt if ctx.needs_input_grad[1] else None), None, None


def equivariance_loss_batch(A, At, theta_inv, nb):
    """(nb,) equivariance losses of nb replicas (T selected rows each, stacked in A / At)."""
    _lib.require_device(A, At)
    if A.shape[0] % nb or theta_inv.numel() != 6 * nb:
        raise ValueError(f"{A.shape[0]} rows / theta_inv {tuple(theta_inv.shape)} for {nb} images")
    return EquivarianceLossBatch.apply(A, At, theta_inv, int(nb))


# --------------------------------------------------------------------------- UNet-side GroupNorm(+SiLU)
# GN_EPI (tests set False to compare): the Winograd convolution's epilogue writes per-segment (mean, M2) of
# its output (skp_conv3x3_wino2_gn) and a GroupNorm reading that output takes its statistics from
# them (skp_groupnorm_fwd_part) instead of a pass over the activation.
GN_EPI = True   # tests switch it: False = GroupNorm computes its own statistics


def _gn_parts_of(x):
    """The (mean, M2) segment partials the producing convolution left on ``x`` (None: none, or x was
    modified in place since)."""
    ent = getattr(x, "_skp_gn", None)
    if ent is None or ent[0] != x._version:
        return None
    return ent[1], ent[2]


def _gn_fwd(x, gamma, beta, shift, groups, eps, act):
    """act(GroupNorm(x + shift)) forward: (y, stats, g, b, nws) — skp_groupnorm_fwd, or
    skp_groupnorm_fwd_part when x carries its producer's statistics partials."""
    B, C = x.shape[:2]
    HW = x[0, 0].numel()
    nws = _lib.lib().skp_groupnorm_workspace(B, C, HW, groups)
    if nws < 0:
        raise ValueError(f"groupnorm: bad shape {tuple(x.shape)} groups={groups}")
    part = torch.empty(nws, device=x.device, dtype=torch.float64)
    stats = torch.empty(B * groups * 2, device=x.device, dtype=F32)
    y = torch.empty_like(x)
    g, b = _c(gamma.detach()), _c(beta.detach())
    pre = _gn_parts_of(x) if GN_EPI else None
    if pre is not None:
        call("skp_groupnorm_fwd_part", ptr(x), ptr(g), ptr(b), ptr(shift), ptr(pre[0]), pre[1], B, C, HW,
             int(groups), float(eps), int(act), ptr(y), ptr(stats), ptr(part), stream(x.device))
    else:
        call("skp_groupnorm_fwd", ptr(x), ptr(g), ptr(b), ptr(shift), B, C, HW, int(groups), float(eps), int(act),
             ptr(y), ptr(stats), ptr(part), stream(x.device))
    return y, stats, g, b, nws


class GroupNormAct(torch.autograd.Function):
    """y = act(GroupNorm(x + shift)) with frozen affine parameters (dx only) — skp_groupnorm_fwd/bwd.
    ``shift`` (B, C) or None: a per-(sample, channel) input offset (conv bias + time embedding)."""

    @staticmethod
    def forward(ctx, x, gamma, beta, groups, eps, act, shift):
        x = _c(x)
        B, C = x.shape[:2]
        HW = x[0, 0].numel()
        if shift is not None:
            shift = _c(shift.detach().expand(B, C))
        y, stats, g, b, nws = _gn_fwd(x, gamma, beta, shift, groups, eps, act)
        ctx.save_for_backward(x, g, b, stats, shift)
        ctx.meta = (B, C, HW, int(groups), int(act), nws)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, g, b, stats, shift = ctx.saved_tensors
        B, C, HW, G, act, nws = ctx.meta
        dy = _c(dy)
        dx = torch.empty_like(x)
        part = torch.empty(nws, device=x.device, dtype=torch.float64)
        call("skp_groupnorm_bwd", ptr(x), ptr(dy), ptr(g), ptr(b), ptr(shift), ptr(stats), B, C, HW, G, act, ptr(dx),
             ptr(part), stream(x.device))
        return dx, None, None, None, None, None, None


class GroupNormActRes(torch.autograd.Function):
    """GroupNormAct that also hands x on (``x_pass``, the same values) to its other consumer — the
    residual or shortcut of a ResNet block / spatial transformer — so that consumer's gradient
    comes back to THIS node and is added inside the backward kernel (skp_groupnorm_bwd_add) instead
    of by a separate autograd accumulation pass over the activation."""

    @staticmethod
    def forward(ctx, x, gamma, beta, groups, eps, act, shift):
        xc = _c(x)
        B, C = xc.shape[:2]
        HW = xc[0, 0].numel()
        if shift is not None:
            shift = _c(shift.detach().expand(B, C))
        y, stats, g, b, nws = _gn_fwd(xc, gamma, beta, shift, groups, eps, act)
        ctx.save_for_backward(xc, g, b, stats, shift)
        ctx.meta = (B, C, HW, int(groups), int(act), nws)
        return y, x.view_as(x)

    @staticmethod
    def backward(ctx, dy, dpass):
        x, g, b, stats, shift = ctx.saved_tensors
        B, C, HW, G, act, nws = ctx.meta
        dy = _c(dy)
        dres = None if dpass is None else _c16(dpass)
        dx = torch.empty_like(x)
        part = torch.empty(nws, device=x.device, dtype=torch.float64)
        call("skp_groupnorm_bwd_add", ptr(x), ptr(dy), ptr(g), ptr(b), ptr(shift), ptr(stats), B, C, HW, G, act,
             ptr(dres), ptr(dx), ptr(part), stream(x.device))
        return dx, None, None, None, None, None, None


def group_norm_act_res(x, gamma, beta, groups, eps, act):
    """(act(GroupNorm(x)), x) where the second output is x for the node's other consumer: its
    gradient is added by the GroupNorm backward kernel (GroupNormActRes)."""
    _lib.require_device(x)
    return GroupNormActRes.apply(x, gamma, beta, int(groups), float(eps), bool(act), None)


def group_norm_act(x, gamma, beta, groups, eps, act, shift=None):
    """Fused GroupNorm(x + shift) (+SiLU when act) on the HIP device; frozen gamma/beta.
    ``shift``: None or a (B, C) / (1, C) / (C,) per-channel input offset without gradient."""
    _lib.require_device(x)
    if shift is not None:
        shift = shift.reshape(-1, x.shape[1]).to(x.device, F32)
    return GroupNormAct.apply(x, gamma, beta, int(groups), float(eps), bool(act), shift)


class ResidualBiasAdd(torch.autograd.Function):
    """out = a + (h + bias[c]) (bias frozen): gradients pass through to a and h."""

    @staticmethod
    def forward(ctx, a, h, bias):
        a, h = _c(a), _c(h)
        B, C = a.shape[:2]
        out = torch.empty_like(a)
        call("skp_residual_bias_add", ptr(a), ptr(h), ptr(_c(bias.detach())), B, C, a[0, 0].numel(), ptr(out),
             stream(a.device))
        return out

    @staticmethod
    def backward(ctx, g):
        return g, g, None


def residual_bias_add(a, h, bias):
    """a + (h + bias[:, None, None]) for NCHW a, h on the HIP device."""
    _lib.require_device(a, h)
    if a.shape != h.shape:
        raise ValueError(f"residual_bias_add: shapes {tuple(a.shape)} and {tuple(h.shape)} differ")
    return ResidualBiasAdd.apply(a, h, bias)


def softmax_(s):
    """In-place row softmax of a contiguous fp32 (…, cols) tensor (skp_softmax_fwd), torch
    semantics; falls back to torch's when cols is not a multiple of 4."""
    if s.dtype != F32 or not s.is_contiguous() or s.shape[-1] % 4 or s.shape[-1] > 16384 or \
            s.data_ptr() % 16:
        return s.copy_(s.softmax(dim=-1))
    call("skp_softmax_fwd", ptr(s), s.numel() // s.shape[-1], s.shape[-1], stream(s.device))
    return s


def attention_probs(q, k, scale):
    """softmax(q kᵀ·scale) for (B·H, S, D) q and (B·H, S', D) k: hipBLASLt baddbmm, then the
    softmax in place (skp_softmax_fwd)."""
    sim = torch.baddbmm(torch.empty(q.shape[0], q.shape[1], k.shape[1], dtype=q.dtype, device=q.device),
                        q, k.transpose(1, 2), beta=0, alpha=scale)
    return softmax_(sim)


def attention_nograd(q, k, v, scale):
    """softmax(q kᵀ·scale) v when no gradient is needed: the fused online-softmax kernel
    (skp_attn_fwd, no score tensor; any key count) where the shapes allow, else the scores +
    in-place softmax."""
    BH, S, d = q.shape
    L = k.shape[1]
    if (q.dtype == F32 and S % 64 == 0 and d in (40, 64, 80) and q.is_contiguous()
            and k.is_contiguous() and v.is_contiguous()):
        out = torch.empty_like(q)
        call("skp_attn_fwd", ptr(q), ptr(k), ptr(v), ptr(out), None, BH, S, L, d, float(scale), stream(q.device))
        return out
    return torch.bmm(attention_probs(q, k, scale), v)


# head dims routed to skp_attn_bwd_kv: d = 40 measured faster end to end (2 waves per SIMD fit);
# d = 64 / 80 run at one wave per SIMD and measured slower than the unfused path.
# (tests route every supported head dim through it, or none)
ATTN_FUSED_KV = (40,)


class MathAttention(torch.autograd.Function):
    """softmax(q kᵀ·scale) v over (B·H, S, D) (diffusers-0.8.0 math path): hipBLASLt GEMMs and
    the in-place skp_softmax_fwd.  Backward: dV = Pᵀ dO (hipBLASLt), then the score gradient
    with baddbmm's scale folded in — one skp_attn_dscore pass over P (dO·Vᵀ on the matrix
    cores, never materialised; D = rowsum(dO ⊙ O)) where the shapes allow, else dP = dO Vᵀ and
    one skp_softmax_bwd pass written over it — then dQ = dS K, dK = dSᵀ Q.  When K needs a
    gradient and d ∈ ATTN_FUSED_KV, skp_attn_bwd_kv produces dS, dV and dK in one pass over P
    (dV, dK accumulated on the matrix cores per key block); only dQ = dS K stays a GEMM."""

    @staticmethod
    def forward(ctx, q, k, v, scale):
        p = attention_probs(q, k, scale)
        out = torch.bmm(p, v)
        ctx.save_for_backward(q, k, v, p, out)
        ctx.scale = scale
        return out

    @staticmethod
    def backward(ctx, dout):
        q, k, v, p, out = ctx.saved_tensors
        dout = dout.contiguous()
        BH, S, L = p.shape
        d = q.shape[2]
        if (d in ATTN_FUSED_KV and S % 64 == 0 and L % 64 == 0 and ctx.needs_input_grad[1]
                and all(t.is_contiguous() and t.data_ptr() % 16 == 0 for t in (q, v, dout))):
            D = (dout * out).sum(-1)
            ds, dv, dk = torch.empty_like(p), torch.empty_like(v), torch.empty_like(k)
            call("skp_attn_bwd_kv", ptr(p), ptr(dout), ptr(q), ptr(v), ptr(D), ptr(ds), ptr(dv), ptr(dk),
                 BH, S, L, d, float(ctx.scale), stream(p.device))
            dq = torch.bmm(ds, k) if ctx.needs_input_grad[0] else None
            return dq, dk, dv if ctx.needs_input_grad[2] else None, None
        dv = torch.bmm(p.transpose(1, 2), dout) if ctx.needs_input_grad[2] else None
        dq = dk = None
        if ctx.needs_input_grad[0] or ctx.needs_input_grad[1]:
            if S % 64 == 0 and L % 64 == 0 and d in (40, 64, 80, 160) and v.is_contiguous():
                D = (dout * out).sum(-1)
                ds = torch.empty_like(p)
                call("skp_attn_dscore", ptr(p), ptr(dout), ptr(v), ptr(D), ptr(ds), BH, S, L, d,
                     float(ctx.scale), stream(p.device))
            else:
                ds = torch.bmm(dout, v.transpose(1, 2))             # dP, overwritten by scale·dS
                call("skp_softmax_bwd", ptr(p), ptr(ds), p.shape[0] * p.shape[1], p.shape[2], float(ctx.scale),
                     stream(p.device))
            dq = torch.bmm(ds, k) if ctx.needs_input_grad[0] else None
            dk = torch.bmm(ds.transpose(1, 2), q) if ctx.needs_input_grad[1] else None
        return dq, dk, dv, None


class LayerNormFn(torch.autograd.Function):
    """LayerNorm over the last dimension with frozen γ, β (input gradient only) —
    skp_layernorm_fwd/bwd, one wave per row."""

    @staticmethod
    def forward(ctx, x, weight, bias, eps):
        x = _c(x)
        C = x.shape[-1]
        rows = x.numel() // C
        y = torch.empty_like(x)
        stats = torch.empty(rows, 2, device=x.device, dtype=F32)
        w, b = _c(weight.detach()), _c(bias.detach())
        call("skp_layernorm_fwd", ptr(x), ptr(w), ptr(b), rows, C, float(eps), ptr(y), ptr(stats), stream(x.device))
        ctx.save_for_backward(x, w, stats)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, w, stats = ctx.saved_tensors
        dy = _c(dy)
        C = x.shape[-1]
        dx = torch.empty_like(x)
        call("skp_layernorm_bwd", ptr(x), ptr(dy), ptr(w), ptr(stats), x.numel() // C, C, ptr(dx), stream(x.device))
        return dx, None, None, None


class LayerNormRes(torch.autograd.Function):
    """LayerNormFn that also hands x on (``x_pass``) to the transformer block's residual add, so the
    residual's gradient is added inside the backward kernel (skp_layernorm_bwd_add) rather than by
    a separate autograd accumulation pass (h = attn(norm(h)) + h, diffusers attention.py)."""

    @staticmethod
    def forward(ctx, x, weight, bias, eps):
        xc = _c(x)
        C = xc.shape[-1]
        rows = xc.numel() // C
        y = torch.empty_like(xc)
        stats = torch.empty(rows, 2, device=xc.device, dtype=F32)
        w, b = _c(weight.detach()), _c(bias.detach())
        call("skp_layernorm_fwd", ptr(xc), ptr(w), ptr(b), rows, C, float(eps), ptr(y), ptr(stats), stream(xc.device))
        ctx.save_for_backward(xc, w, stats)
        return y, x.view_as(x)

    @staticmethod
    def backward(ctx, dy, dpass):
        x, w, stats = ctx.saved_tensors
        dy = _c(dy)
        dres = None if dpass is None else _c16(dpass)
        C = x.shape[-1]
        dx = torch.empty_like(x)
        call("skp_layernorm_bwd_add", ptr(x), ptr(dy), ptr(w), ptr(stats), x.numel() // C, C, ptr(dres), ptr(dx),
             stream(x.device))
        return dx, None, None, None


def layer_norm_res(x, weight, bias, eps):
    """(F.layer_norm(x, …), x) with the second output for the residual add: its gradient joins the
    LayerNorm backward kernel (LayerNormRes).  Shapes the kernel does not take: torch's LayerNorm
    and x itself."""
    _lib.require_device(x)
    C = x.shape[-1]
    if (x.dtype != F32 or C % 4 or C > 2048 or weight is None or bias is None or weight.requires_grad
            or bias.requires_grad or x.numel() == 0 or x.numel() // C < LN_MIN_ROWS):
        return torch.nn.functional.layer_norm(x, (C,), weight, bias, eps), x
    return LayerNormRes.apply(x, weight, bias, float(eps))


# kernel time at batch 8 (tools/ln_time.py): 32768 rows × 320: 15.4 µs = 5.4 TB/s (ATen 40.8);
# 8192 × 640: 7.6 (13.8); 2048 × 1280: 7.1 (7.5).  Fewer rows than this stay on ATen.
LN_MIN_ROWS = 2048


def layer_norm(x, weight, bias, eps):
    """F.layer_norm(x, (C,), weight, bias, eps) with frozen affine parameters on the HIP device
    (skp_layernorm_*) for ≥ LN_MIN_ROWS rows; torch's form for fewer rows, other dtypes / widths."""
    _lib.require_device(x)
    C = x.shape[-1]
    if (x.dtype != F32 or C % 4 or C > 2048 or weight is None or bias is None or weight.requires_grad
            or bias.requires_grad or x.numel() == 0 or x.numel() // C < LN_MIN_ROWS):
        return torch.nn.functional.layer_norm(x, (C,), weight, bias, eps)
    return LayerNormFn.apply(x, weight, bias, float(eps))


class Geglu(torch.autograd.Function):
    """x · gelu(gate) over the two halves of a (…, 2I) projection (diffusers GEGLU): one fused
    pass each way (skp_geglu_fwd / skp_geglu_bwd)."""

    @staticmethod
    def forward(ctx, h):
        h = _c(h)
        I = h.shape[-1] // 2
        out = torch.empty(*h.shape[:-1], I, device=h.device, dtype=F32)
        call("skp_geglu_fwd", ptr(h), h.numel() // h.shape[-1], I, ptr(out), stream(h.device))
        ctx.save_for_backward(h)
        return out

    @staticmethod
    def backward(ctx, dout):
        (h,) = ctx.saved_tensors
        dout = _c(dout)
        dh = torch.empty_like(h)
        call("skp_geglu_bwd", ptr(h), ptr(dout), h.numel() // h.shape[-1], h.shape[-1] // 2, ptr(dh),
             stream(h.device))
        return dh


def geglu(h):
    """diffusers GEGLU's `x, gate = h.chunk(2, -1); x * gelu(gate)` (exact GELU) on the HIP
    device; torch's form where the half width is not a multiple of 4."""
    _lib.require_device(h)
    if h.dtype != F32 or h.shape[-1] % 8:
        x, gate = h.chunk(2, dim=-1)
        return x * torch.nn.functional.gelu(gate)
    return Geglu.apply(h)


# head dims whose grad-needing attention keeps no probability tensor (FlashAttention below);
# (tests route every supported head dim through it, or none)
ATTN_FLASH = (40, 64)


class FlashAttention(torch.autograd.Function):
    """softmax(q kᵀ·scale) v without a saved (B·H, S, L) probability tensor: the forward is the
    online-softmax skp_attn_fwd emitting per-row (max, 1/sum); the backward skp_attn_bwd_flash
    rebuilds P per key block from q kᵀ and those stats and produces dS, dV, dK in one pass
    (dQ = dS k stays a GEMM).  Same result as MathAttention within fp32 rounding."""

    @staticmethod
    def forward(ctx, q, k, v, scale):
        BH, S, d = q.shape
        L = k.shape[1]
        out = torch.empty_like(q)
        stats = torch.empty(BH, S, 2, device=q.device, dtype=F32)
        call("skp_attn_fwd", ptr(q), ptr(k), ptr(v), ptr(out), ptr(stats), BH, S, L, d, float(scale),
             stream(q.device))
        ctx.save_for_backward(q, k, v, out, stats)
        ctx.scale = scale
        return out

    @staticmethod
    def backward(ctx, dout):
        q, k, v, out, stats = ctx.saved_tensors
        dout = dout.contiguous()
        BH, S, d = q.shape
        L = k.shape[1]
        D = (dout * out).sum(-1)
        ds = torch.empty(BH, S, L, device=q.device, dtype=F32)
        dv, dk = torch.empty_like(v), torch.empty_like(k)
        call("skp_attn_bwd_flash", ptr(q), ptr(k), ptr(v), ptr(dout), ptr(stats), ptr(D), ptr(ds), ptr(dv), ptr(dk),
             BH, S, L, d, float(ctx.scale), stream(q.device))
        dq = torch.bmm(ds, k) if ctx.needs_input_grad[0] else None
        return dq, dk if ctx.needs_input_grad[1] else None, dv if ctx.needs_input_grad[2] else None, None


def math_attention(q, k, v, scale):
    """softmax(q kᵀ·scale) v with a fused backward (HIP device): FlashAttention for the head
    dims in ATTN_FLASH when S is a multiple of 64 (any key count: the last key block is
    masked), else MathAttention."""
    _lib.require_device(q, k, v)
    BH, S, d = q.shape
    L = k.shape[1]
    if (d in ATTN_FLASH and S % 64 == 0 and q.dtype == F32
            and all(t.dtype == F32 and t.is_contiguous() and t.data_ptr() % 16 == 0 for t in (q, k, v))):
        return FlashAttention.apply(q, k, v, float(scale))
    return MathAttention.apply(q, k, v, float(scale))


# --------------------------------------------------------------------------- attention on (B, S, H·d) projections
# A/B: 0 = permute q / k / v / out between (B, S, H·d) and (B·H, S, d) around the attention kernels (r02)
ATTN_BSHD = True


def _lay(t):
    """(batch stride, row stride) of a (B, S, H·d) operand whose last dimension is unit-stride."""
    return int(t.stride(0)), int(t.stride(1))


def _bshd_ok(q, k, v, H):
    B, S, C = q.shape
    if not ATTN_BSHD or C % H or S % 64 or k.shape[-1] != C or v.shape[-1] != C:
        return False
    return all(t.is_cuda and t.dtype == F32 and t.dim() == 3 and t.stride(2) == 1 and t.stride(1) % 4 == 0
               and t.stride(0) % 4 == 0 and t.data_ptr() % 16 == 0 for t in (q, k, v))


class FlashAttentionBSHD(torch.autograd.Function):
    """FlashAttention on the projections' own (B, S, H·d) layout: skp_attn_fwd_bshd reads q / k / v
    and writes the output with head strides (no reshape_heads_to_batch_dim / _to_heads copies, a
    batch-shared k / v read through a zero batch stride), skp_attn_bwd_flash_bshd reads dO, q, k, v
    the same way and writes dV, dK per image in (B, L, H·d) (summed over a shared batch by the
    expand's backward).  dQ = dS·K is one torch.matmul per head (its operands are the only permutes
    left)."""

    @staticmethod
    def forward(ctx, q, k, v, H, scale):
        B, S, C = q.shape
        L = k.shape[1]
        d = C // H
        out = torch.empty(B, S, C, device=q.device, dtype=F32)
        stats = torch.empty(B * H, S, 2, device=q.device, dtype=F32)
        call("skp_attn_fwd_bshd", ptr(q), *_lay(q), ptr(k), *_lay(k), ptr(v), *_lay(v), ptr(out), S * C, C, ptr(stats),
             B, H, S, L, d, float(scale), stream(q.device))
        ctx.save_for_backward(q, k, v, out, stats)
        ctx.H, ctx.scale = H, scale
        return out

    @staticmethod
    def backward(ctx, dout):
        q, k, v, out, stats = ctx.saved_tensors
        H, scale = ctx.H, ctx.scale
        dout = _c16(dout)
        B, S, C = q.shape
        L = k.shape[1]
        d = C // H
        D = (dout.view(B, S, H, d) * out.view(B, S, H, d)).sum(-1).transpose(1, 2).contiguous()   # (B, H, S)
        ds = torch.empty(B * H, S, L, device=q.device, dtype=F32)
        dv = torch.empty(B, L, C, device=q.device, dtype=F32)
        dk = torch.empty(B, L, C, device=q.device, dtype=F32)
        call("skp_attn_bwd_flash_bshd", ptr(q), *_lay(q), ptr(k), *_lay(k), ptr(v), *_lay(v), ptr(dout), S * C, C,
             ptr(stats), ptr(D), ptr(ds), ptr(dv), L * C, C, ptr(dk), L * C, C, B, H, S, L, d, float(scale),
             stream(q.device))
        dq = None
        if ctx.needs_input_grad[0]:
            k4 = k.view(k.shape[0], L, H, d).transpose(1, 2).expand(B, H, L, d)
            dq = torch.matmul(ds.view(B, H, S, L), k4).transpose(1, 2).reshape(B, S, C)
        return (dq, dk if ctx.needs_input_grad[1] else None, dv if ctx.needs_input_grad[2] else None, None, None)


def attention_heads(q, k, v, H, scale):
    """softmax(q kᵀ·scale) v per head for (B, S, H·d) q and (B or stride-0 B, L, H·d) k, v, output
    (B, S, H·d) — diffusers' CrossAttention between to_q/to_k/to_v and to_out without the head
    permutes.  None when the shape is not covered (the caller keeps the permuting path): the
    gradient-needing form for a batch-shared context and head dims in ATTN_FLASH, the no-grad
    online-softmax form for d ∈ {40, 64, 80}, S a multiple of 64."""
    if not _bshd_ok(q, k, v, H):
        return None
    B, S, C = q.shape
    d = C // H
    if torch.is_grad_enabled() and (q.requires_grad or k.requires_grad or v.requires_grad):
        # gradient-needing self-attention keeps the head-major copies: both kernels re-read K / V once
        # per 64-row block, and a head's 160-B rows strided by H·d touch 1.6× the cache lines; at the
        # 64² shape that costs more than the permutes (measured: 2.05 + 3.85 ms vs 1.85 + 3.38 ms for
        # the kernels, tools/attn_bshd_time.py); a batch-shared context (cross-attention) is small and
        # takes this path (0.95 vs 1.00 ms per call)
        if d not in ATTN_FLASH or k.stride(0) != 0:
            return None
        return FlashAttentionBSHD.apply(q, k, v, int(H), float(scale))
    if d not in (40, 64, 80):
        return None
    out = torch.empty(B, S, C, device=q.device, dtype=F32)
    call("skp_attn_fwd_bshd", ptr(q), *_lay(q), ptr(k), *_lay(k), ptr(v), *_lay(v), ptr(out), S * C, C, None,
         B, H, S, k.shape[1], d, float(scale), stream(q.device))
    return out


# --------------------------------------------------------------------------- UNet-side: token projections
_QKV_W = {}   # (id wq, id wk, id wv) -> ((versions), weakref(wq), [wq; wk; wv])


def _qkv_weight(*ws):
    """[w0; w1; …] of frozen projection weights, built once per weight set (and its versions): the
    entry is reused only while EVERY weight is still the object it was built from (a weakref per
    weight, so a replaced to_k / to_v never meets a stale concatenation through a reused id) with
    the same storage and version; it is dropped when any of them is collected."""
    key = tuple(id(w) for w in ws)
    sig = tuple((w._version, w.data_ptr()) for w in ws)
    ent = _QKV_W.get(key)
    if ent is not None and ent[0] == sig and all(r() is w for r, w in zip(ent[1], ws)):
        return ent[2]
    w3 = torch.cat([w.detach() for w in ws], 0).contiguous()
    drop = lambda _r, key=key: _QKV_W.pop(key, None)   # noqa: E731
    _QKV_W[key] = (sig, tuple(_weakref.ref(w, drop) for w in ws), w3)
    return w3


class QKVProjection(torch.autograd.Function):
    """q, k, v = to_q(x), to_k(x), to_v(x) of a self-attention (diffusers CrossAttention with
    context = x, bias-free, frozen) as ONE GEMM against [Wq; Wk; Wv] (x read once; q, k, v are
    column views of the (B, S, 3C) product).  Backward: dx = dq Wq, then dk Wk and dv Wv
    accumulated into it by the GEMM (beta = 1): no separate gradient-sum passes over dx."""

    @staticmethod
    def forward(ctx, x, w3, C):
        out = torch.matmul(x, w3.t())
        ctx.save_for_backward(w3)
        ctx.C = C
        ctx.x_shape = x.shape
        ctx.set_materialize_grads(False)   # an unused projection's gradient stays None (skipped)
        return tuple(out[..., i * C:(i + 1) * C] for i in range(w3.shape[0] // C))

    @staticmethod
    def backward(ctx, *grads):
        (w3,) = ctx.saved_tensors
        C = ctx.C
        dx = None
        for i, g in enumerate(grads):
            if g is None:
                continue
            g2 = g.reshape(-1, C)
            wi = w3[i * C:(i + 1) * C]
            if dx is None:
                dx = torch.mm(g2, wi)
            else:
                dx.addmm_(g2, wi)
        if dx is None:   # no projection received a gradient
            return None, None, None
        return dx.view(ctx.x_shape), None, None


# (QKV_FUSED = False: three nn.Linear calls and autograd's gradient sum)
QKV_FUSED = True


def qkv_projection(x, *ws):
    """(x W0ᵀ, x W1ᵀ, …) of bias-free projections with equal output widths on the HIP device in
    one GEMM (QKVProjection): q, k, v of a self-attention, or k, v of the shared context."""
    _lib.require_device(x)
    return QKVProjection.apply(x, _qkv_weight(*ws), int(ws[0].shape[0]))


class TokensProjIn(torch.autograd.Function):
    """Transformer2DModel.proj_in (1×1 conv) + NCHW→(B, HW, C') as ONE strided batched GEMM:
    h[b] = x[b]ᵀ Wᵀ + bias, x (B, C, HW) read through a transposed view (no permute copy, no
    NHWC conversion); the input gradient comes back in NCHW the same way (W frozen)."""

    @staticmethod
    def forward(ctx, x, w, bias):
        B, C, HW = x.shape
        h = torch.bmm(x.transpose(1, 2), w.t().expand(B, C, w.shape[0]))
        if bias is not None:
            h.add_(bias)
        ctx.save_for_backward(w)
        return h

    @staticmethod
    def backward(ctx, dh):
        (w,) = ctx.saved_tensors
        B = dh.shape[0]
        dx = torch.bmm(w.t().expand(B, w.shape[1], w.shape[0]), dh.transpose(1, 2))   # (B, C, HW)
        return dx, None, None


class TokensProjOut(torch.autograd.Function):
    """Transformer2DModel.proj_out (1×1 conv) on (B, HW, C') tokens back to NCHW as one strided
    batched GEMM, y[b] = W h[b]ᵀ; the bias and the residual follow in one residual_bias_add."""

    @staticmethod
    def forward(ctx, h, w):
        B = h.shape[0]
        ctx.save_for_backward(w)
        return torch.bmm(w.expand(B, *w.shape), h.transpose(1, 2))                     # (B, C, HW)

    @staticmethod
    def backward(ctx, dy):
        (w,) = ctx.saved_tensors
        B = dy.shape[0]
        return torch.bmm(dy.transpose(1, 2), w.expand(B, *w.shape)), None             # (B, HW, C')


def tokens_proj_in(x, weight, bias):
    """(B, C, H, W) → (B, HW, C') = 1×1 conv (weight (C', C, 1, 1)) + bias, flattened to tokens."""
    B, C = x.shape[:2]
    return TokensProjIn.apply(x.reshape(B, C, -1), weight.detach().reshape(weight.shape[0], C),
                              None if bias is None else bias.detach())


def tokens_proj_out(h, weight, bias, residual):
    """(B, HW, C') → residual + 1×1 conv(h) + bias in NCHW (residual's shape)."""
    B, C = residual.shape[:2]
    y = TokensProjOut.apply(h, weight.detach().reshape(C, h.shape[-1]))
    return residual_bias_add(residual, y.view(residual.shape), bias)


# --------------------------------------------------------------------------- 3×3 convolution
# Transformed weights per frozen weight tensor: {weight: {flip: (version, U)}} (U = G g Gᵀ,
# K·C·36 floats; built once, on first use, on the weight's device and stream).
import weakref as _weakref

_WINO_U = {}   # id(weight) -> (weakref(weight), {(flip, v2): (version, U)})
# Shapes whose grid stays below this even after splitting go to MIOpen.
WINO_MIN_WORKGROUPS = 128
# Which kernel takes an eligible shape: "auto" = skp_conv3x3_wino2 where H and W are multiples
# of 32 (every VAE-encoder layer, the UNet's 64² and 32² layers) or 16×16 with the batch a
# multiple of 4 (the UNet's 16² layers), skp_conv3x3_wino elsewhere (8²);
# "v1" forces the first kernel (tests).  WINO_SPLIT = False disables split-K; WINO_NSPLIT_FORCE
# (tests, tools/wino_time.py) measures one given split.
WINO_KERNEL = "auto"
WINO_SPLIT = True
WINO_NSPLIT_FORCE = 0


def _wino_v2(H, W, B=None):
    """skp_conv3x3_wino2 takes H, W multiples of 32, and 16×16 images four at a time."""
    if WINO_KERNEL == "v1":
        return False
    return (H % 32 == 0 and W % 32 == 0) or (H == 16 and W == 16 and B is not None and B % 4 == 0)


def _wino_u(weight, flip, v2=False):
    ent = _WINO_U.get(id(weight))
    if ent is None or ent[0]() is not weight:
        key = id(weight)
        ent = (_weakref.ref(weight, lambda _r, key=key: _WINO_U.pop(key, None)), {})
        _WINO_U[key] = ent
    per = ent[1]
    hit = per.get((flip, v2))
    if hit is not None and hit[0] == weight._version:
        return hit[1]
    w = _c(weight.detach())
    K, C = (w.shape[0], w.shape[1]) if not flip else (w.shape[1], w.shape[0])
    U = torch.empty(K * C * (40 if v2 else 36), device=w.device, dtype=F32)
    call("skp_wino2_weights" if v2 else "skp_wino_weights", ptr(w), K, C, int(flip), ptr(U), stream(w.device))
    per[(flip, v2)] = (weight._version, U)
    return U


def _wino_plan_uncached(B, C, K, H, W, force):
    """(v2, nsplit, workgroups) for a (B, C, H, W) → (B, K, H, W) convolution.

    One workgroup per CU (their LDS), so a grid runs in ceil(workgroups / 256) rounds of
    (stages × ≈2.4 µs + ≈5 µs); splitting the input channels S ways shortens a workgroup S-fold
    and adds (S + 1) passes over the output for the partial sums.  The split with the least
    modelled time wins (measured at batch 8: 64² × 320 and 32² × 640 channels at 4 and 8 splits
    instead of 1.25 and 0.63 rounds)."""
    v2 = _wino_v2(H, W, B)
    if v2:
        wgs = (B // 4 if H == 16 else B * (H // 32) * (W // 32)) * (K // 32)
    elif B * (H // 4) * (W // 4) <= 32 and K % 64 == 0:
        wgs = K // 64   # one 32-tile × 64-channel block per channel block (libskp's rule, skp_conv.hip)
    else:
        wgs = -(-(B * (H // 4) * (W // 4)) // 64) * (K // 32)
    out_bytes = B * K * H * W * 4
    half = v2   # libskp's half-height blocks: two co-resident workgroups per CU

    def cost(s):
        if half:
            # half-height blocks (2·wgs workgroups, two co-resident per CU): a CU holding k of them
            # runs ⌊k/2⌋ pairs at ≈1.72 µs per stage and a lone one at ≈1.48; the partial sums
            # cost (s + 1) passes at ≈2 TB/s (fitted to the split sweep, profiles/r03am_split_sweep.txt)
            k = -(-2 * wgs * s // 256)
            st = C // s // 4
            return (k // 2) * st * 1.72e-6 + (k % 2) * st * 1.48e-6 + (s > 1) * (s + 1) * out_bytes / 2e12
        rounds = -(-wgs * s // 256)
        return rounds * ((C // s // 4) * 2.4e-6 + 5e-6) + (s > 1) * (s + 1) * out_bytes / 5e12

    nsplit = 1
    if WINO_SPLIT:
        cands = [s for s in range(1, 33) if C % (4 * s) == 0 and (s == 1 or C // s >= 32)]
        nsplit = min(cands, key=cost)
        if force and C % (4 * force) == 0:   # dev: WINO_NSPLIT_FORCE measures a given split
            nsplit = force
    return v2, nsplit, wgs * nsplit


_WINO_PLANS = {}


def _wino_plan(B, C, K, H, W):
    """_wino_plan_uncached, memoised per shape (and the module switches it reads): the planner's
    32-candidate cost loop ran in Python on every convolution call, ~1500 launches per step."""
    force = int(WINO_NSPLIT_FORCE)
    key = (B, C, K, H, W, force, WINO_KERNEL, WINO_SPLIT)
    plan = _WINO_PLANS.get(key)
    if plan is None:
        plan = _WINO_PLANS[key] = _wino_plan_uncached(B, C, K, H, W, force)
    return plan


def wino_eligible(B, C, K, H, W, min_workgroups=None):
    """Whether a Winograd kernel takes a (B, C, H, W) → (B, K, H, W) 3×3 convolution."""
    if C % 4 or K % 32 or H % 4 or W % 4:
        return False
    wgs = _wino_plan(B, C, K, H, W)[2]
    return wgs >= (WINO_MIN_WORKGROUPS if min_workgroups is None else min_workgroups)


# Small-image, many-channel convolutions (the UNet's 8²-32² layers) as Winograd transforms + 36
# batched library GEMMs (skp_wino_in_transform → torch.bmm → skp_wino_out_transform) instead of the
# fused kernels: at these sizes the fused grids are a few hundred latency-bound workgroups.
# WINO_GEMM_MAX_HW = the largest H·W that takes it (tests set 0 to cover the fused kernels).
WINO_GEMM_MAX_HW = 1024
WINO_GEMM_MIN_CH = 256
# G of F(4×4, 3×3) at the points (0, 1, −1, 1/2, −2, ∞) (skp_conv.hip wino_weights_kernel's Gm)
_WINO_G = ((1.0, 0.0, 0.0), (1 / 3, 1 / 3, 1 / 3), (-1 / 3, 1 / 3, -1 / 3), (-16 / 15, -8 / 15, -4 / 15),
           (1 / 15, -2 / 15, 4 / 15), (0.0, 0.0, 1.0))


def _wino_gemm_ok(B, C, K, H, W):
    return (0 < H * W <= WINO_GEMM_MAX_HW and C >= WINO_GEMM_MIN_CH and K >= WINO_GEMM_MIN_CH
            and H % 4 == 0 and W % 4 == 0 and B * (H // 4) * (W // 4) <= 65535)


def _wino_u_gemm(weight, flip):
    """U[p = 6i + j] (36, C, K) = (G g Gᵀ)[i][j] in fp64 → fp32, g = w[k][c] (flip 0) or
    rot180(w[c][k]) (flip 1, the input-gradient convolution); cached per frozen weight like
    _wino_u."""
    ent = _WINO_U.get(id(weight))
    if ent is None or ent[0]() is not weight:
        key = id(weight)
        ent = (_weakref.ref(weight, lambda _r, key=key: _WINO_U.pop(key, None)), {})
        _WINO_U[key] = ent
    hit = ent[1].get((flip, "gemm"))
    if hit is not None and hit[0] == weight._version:
        return hit[1]
    w = weight.detach().double()
    g = w.flip(2, 3).transpose(0, 1) if flip else w                 # (K, C, 3, 3) of this convolution
    G = torch.tensor(_WINO_G, dtype=torch.float64, device=w.device)
    U = torch.einsum("iu,kcuv,jv->ijck", G, g, G).reshape(36, g.shape[1], g.shape[0]).float().contiguous()
    ent[1][(flip, "gemm")] = (weight._version, U)
    return U


# The product as (36, K, T), so the output transform reads it and writes the tiles coalesced (and
# leaves the next GroupNorm's statistics partials, as the fused kernel does); r04 measured it ahead
# of the (36, T, K) product with per-lane scattered tile stores (skp_wino_out_transform, kept in
# the ABI).


def _wino_gemm_conv(x, weight, flip, bias, residual, K, gn=False):
    B, C, H, W = x.shape
    T = B * (H // 4) * (W // 4)
    U = _wino_u_gemm(weight, flip)
    V = torch.empty(36, C, T, device=x.device, dtype=F32)
    call("skp_wino_in_transform", ptr(x), B, C, H, W, ptr(V), stream(x.device))
    y = torch.empty(B, K, H, W, device=x.device, dtype=F32)
    bp, rp = ptr(bias) if bias is not None else None, ptr(residual) if residual is not None else None
    M = torch.bmm(U.transpose(1, 2), V)                              # (36, K, T)
    P = (H // 4) * (W // 4)
    gnp = None
    if gn and GN_EPI and (P in (16, 32) or P % 64 == 0):
        nseg = P // min(P, 64)
        gnp = torch.empty(B, K, nseg, 2, device=x.device, dtype=F32)
    call("skp_wino_out_transform_kt", ptr(M), B, K, H, W, bp, rp, ptr(y), ptr(gnp), stream(x.device))
    if gnp is not None:
        y._skp_gn = (y._version, gnp, gnp.shape[2])
    return y


def _wino_conv(x, weight, flip, bias, residual, K, gn=False):
    """``gn``: also leave the output's GroupNorm statistics partials on it (``y._skp_gn``) where the
    kernel can write them (skp_conv3x3_wino2_gn: one split, H and W multiples of 32)."""
    B, C, H, W = x.shape
    if _wino_gemm_ok(B, C, K, H, W):
        return _wino_gemm_conv(x, weight, flip, bias, residual, K, gn)
    y = torch.empty(B, K, H, W, device=x.device, dtype=F32)
    # the kernels address x through 32-bit buffer offsets: batches above 2 GiB run in chunks
    per_img = C * H * W * 4
    bmax = max(1, (2 ** 31 - 1) // per_img)
    gnp = None
    if gn and GN_EPI and H % 32 == 0 and W % 32 == 0 and all(
            _wino_plan(min(B, b0 + bmax) - b0, C, K, H, W)[:2] == (True, 1) for b0 in range(0, B, bmax)):
        nseg = (H // 16) * (W // 32)
        gnp = torch.empty(B, K, nseg, 2, device=x.device, dtype=F32)
    for b0 in range(0, B, bmax):
        b1 = min(B, b0 + bmax)
        _wino_launch(x[b0:b1], weight, flip, bias, None if residual is None else residual[b0:b1], y[b0:b1], K,
                     None if gnp is None else gnp[b0:b1])
    if gnp is not None:
        y._skp_gn = (y._version, gnp, gnp.shape[2])
    return y


def _wino_launch(x, weight, flip, bias, residual, y, K, gnp=None):
    B, C, H, W = x.shape
    v2, nsplit, _ = _wino_plan(B, C, K, H, W)
    U = _wino_u(weight, flip, v2)
    ws = torch.empty(nsplit, B, K, H, W, device=x.device, dtype=F32) if nsplit > 1 else None
    name = "skp_conv3x3_wino2" if v2 else "skp_conv3x3_wino"
    args = (ptr(x), ptr(U), ptr(bias) if bias is not None else None,
            ptr(residual) if residual is not None else None, ptr(y), B, C, K, H, W, nsplit,
            ptr(ws) if ws is not None else None)
    with _timed(name, 0):
        if gnp is not None:
            call("skp_conv3x3_wino2_gn", *args, ptr(gnp), stream(x.device))
        else:
            call(name, *args, stream(x.device))


class Conv3x3(torch.autograd.Function):
    """y = conv2d(x, w, bias, padding=1) (+ residual) with a frozen 3×3 weight; the input
    gradient is the same Winograd kernel on the flipped weight (MIOpen when its shape is not
    eligible).  Gradients: x and residual only."""

    @staticmethod
    def forward(ctx, x, weight, bias, residual):
        x = _c(x)
        K = weight.shape[0]
        y = _wino_conv(x, weight, False, None if bias is None else _c(bias.detach()),
                       None if residual is None else _c(residual), K, gn=True)
        ctx.weight = weight
        ctx.xshape = x.shape
        ctx.has_res = residual is not None
        return y

    @staticmethod
    def backward(ctx, dy):
        w = ctx.weight
        B, C, H, W = ctx.xshape
        K = w.shape[0]
        dx = None
        if ctx.needs_input_grad[0]:
            dy = _c(dy)
            if wino_eligible(B, K, C, H, W):
                dx = _wino_conv(dy, w, True, None, None, C)
            else:
                dx = torch.nn.grad.conv2d_input(ctx.xshape, w.detach(), dy, padding=1)
        return dx, None, None, (dy if ctx.has_res else None)


class Conv1x1(torch.autograd.Function):
    """y[b] = W x[b] for a frozen 1×1 convolution (K, C) on NCHW x viewed as (B, C, H·W): ONE strided
    batched GEMM with the weight broadcast over the batch (zero batch stride), straight between NCHW
    tensors — no NCHW↔NHWC transposes around a MIOpen 1×1 kernel; dx[b] = Wᵀ dy[b] the same way."""

    @staticmethod
    def forward(ctx, x, w):
        B, C, H, W = x.shape
        K = w.shape[0]
        y = torch.bmm(w.expand(B, K, C), x.reshape(B, C, H * W))
        ctx.save_for_backward(w)
        ctx.shape = (B, C, H, W)
        return y.view(B, K, H, W)

    @staticmethod
    def backward(ctx, dy):
        (w,) = ctx.saved_tensors
        B, C, H, W = ctx.shape
        K = w.shape[0]
        dx = torch.bmm(w.t().expand(B, C, K), dy.reshape(B, K, H * W)) if ctx.needs_input_grad[0] else None
        return (None if dx is None else dx.view(B, C, H, W)), None


# A/B (default off): 1 = the resnets' 1×1 shortcuts as Conv1x1's batched GEMM.  Measured at the
# bench's shortcut shapes (tools/conv1x1_time.py, batch 8, fwd + input grad): within ±3% of MIOpen's
# 1×1 kernels at 8², 16² and 32² (2560→1280 @16²: 274 vs 272 us; 960→640 @32²: 186 vs 201 us;
# 1280→640 @32²: 290 vs 249 us), the VAE's 128→256 @256² 318 vs 343 us — no net gain, so MIOpen stays
CONV1X1_GEMM = False   # tests switch it: True = 1×1 shortcuts as one GEMM (measured neutral)


def conv1x1(x, weight):
    """Bias-free 1×1 convolution of NCHW fp32 x with a frozen weight (K, C, 1, 1) (the caller folds
    the bias into the next epilogue): Conv1x1's batched GEMM, or F.conv2d with CONV1X1_GEMM off."""
    _lib.require_device(x)
    if weight.requires_grad:
        raise ValueError("conv1x1: the weight must be frozen (requires_grad=False)")
    if not CONV1X1_GEMM or x.dtype != F32:
        return torch.nn.functional.conv2d(x, weight)
    return Conv1x1.apply(_c(x), weight.detach().reshape(weight.shape[0], weight.shape[1]))


# A/B: 0 = the VAE's stride-2 downsampling convolutions run as F.pad + MIOpen (r02)
WINO_S2 = True
WINO_S2_MIN_PIXELS = 384 * 384   # 256² / 128² measured neutral on the copy-free kernel (profiles/r05y_s2_wino_ab.txt)


def conv3x3_s2_eligible(x, weight):
    B, C, H, W = x.shape
    K = weight.shape[0]
    # measured at batch 8 (tools/conv_s2_time.py): 512² × 128 ch 2.21 vs 2.75 ms for pad + MIOpen; at
    # 256² × 256 (1.89 vs 1.85) and 128² × 512 (1.81 vs 1.53) MIOpen's implicit GEMM is as fast or
    # faster than the 4×-redundant Winograd blocks, so only the large-image levels take this path
    return (WINO_S2 and x.is_cuda and x.dtype == F32 and tuple(weight.shape[1:]) == (C, 3, 3) and C % 4 == 0
            and K % 32 == 0 and H % 32 == 0 and W % 32 == 0 and H * W >= WINO_S2_MIN_PIXELS
            and not weight.requires_grad and not (torch.is_grad_enabled() and x.requires_grad))


def conv3x3_s2(x, weight, bias=None):
    """diffusers' Downsample2D(padding=0) — F.pad(x, (0, 1, 0, 1)) then a 3×3 / stride-2 conv2d —
    forward only (the frozen VAE encoder runs without gradient): skp_conv3x3s2_wino2, the stride-1
    pad-1 Winograd convolution sampled at the odd rows / columns (the same taps, the same zero
    row / column past the bottom-right edge) with the bias in its epilogue.  (B, C, H, W) →
    (B, K, H/2, W/2)."""
    _lib.require_device(x)
    if not conv3x3_s2_eligible(x, weight):
        raise ValueError(f"conv3x3_s2: unsupported x {tuple(x.shape)} / weight {tuple(weight.shape)}")
    x = _c16(x)
    B, C, H, W = x.shape
    K = weight.shape[0]
    y = torch.empty(B, K, H // 2, W // 2, device=x.device, dtype=F32)
    U = _wino_u(weight, False, True)
    b = None if bias is None else _c(bias.detach())
    bmax = max(1, (2 ** 31 - 1) // (C * H * W * 4))   # 32-bit buffer offsets into x
    for b0 in range(0, B, bmax):
        b1 = min(B, b0 + bmax)
        _, nsplit, _ = _wino_plan(b1 - b0, C, K, H, W)
        ws = torch.empty(nsplit, b1 - b0, K, H // 2, W // 2, device=x.device, dtype=F32) if nsplit > 1 else None
        with _timed("skp_conv3x3s2_wino2", 0):
            call("skp_conv3x3s2_wino2", ptr(x[b0:b1]), ptr(U), ptr(b), ptr(y[b0:b1]), b1 - b0, C, K, H, W, nsplit,
                 ptr(ws), stream(x.device))
    return y


def conv3x3(x, weight, bias=None, residual=None):
    """3×3 / stride 1 / pad 1 convolution (+ bias, + residual) of NCHW fp32 ``x`` with a frozen
    ``weight`` (K, C, 3, 3): the Winograd F(4×4, 3×3) kernel when the shape is eligible, else
    MIOpen (F.conv2d) with the bias and residual added after."""
    _lib.require_device(x)
    if weight.requires_grad:
        raise ValueError("conv3x3: the weight must be frozen (requires_grad=False)")
    B, C, H, W = x.shape
    K = weight.shape[0]
    if tuple(weight.shape[1:]) != (C, 3, 3):
        raise ValueError(f"conv3x3: weight {tuple(weight.shape)} does not fit input {tuple(x.shape)}")
    if residual is not None and tuple(residual.shape) != (B, K, H, W):
        raise ValueError(f"conv3x3: residual {tuple(residual.shape)} is not ({B}, {K}, {H}, {W})")
    if C % 4 and C < 16 and x.dtype == F32 and wino_eligible(B, C + 4 - C % 4, K, H, W):
        # input layers (RGB: 3 channels): one zero channel makes them Winograd-eligible; the
        # padded weight's transform is rebuilt per call (K·4 entries)
        pad = 4 - C % 4
        xp = torch.nn.functional.pad(x, (0, 0, 0, 0, 0, pad))
        wp = torch.nn.functional.pad(weight.detach(), (0, 0, 0, 0, 0, pad))
        return Conv3x3.apply(xp, wp, bias, residual)
    if x.dtype != F32 or not wino_eligible(B, C, K, H, W):
        y = torch.nn.functional.conv2d(x, weight, bias, 1, 1)
        return y if residual is None else residual + y
    return Conv3x3.apply(x, weight, bias, residual)
