"""Self-contained Stable-Diffusion-1.5 UNet (diffusers-0.8.0 module names) in plain PyTorch.

The reference loads ``UNet2DConditionModel`` from diffusers 0.8.0 through
``StableDiffusionPipeline.from_pretrained`` (reference
``unsupervised_keypoints/optimize_token.py:38-40``).  diffusers is not available
here, so this file restates the SD-1.5 UNet architecture with the same
sub-module names, so a diffusers-0.8.0 ``state_dict`` loads with
``load_state_dict(strict=True)``.  The UNet is frozen on the hot path and stays
in PyTorch-ROCm (fp32); only the attention-capture path is replaced by HIP
kernels (see ``stablekeypoints_amd/ptp_utils.py``).

The hot-path hook walks ``model.named_children()`` for names containing "up"
and patches modules whose class name is exactly ``CrossAttention``
(reference ``ptp_utils.py:555-573``), so that class name and its attribute
interface (``heads``, ``scale``, ``to_q``/``to_k``/``to_v``/``to_out``,
``reshape_heads_to_batch_dim``, ``reshape_batch_dim_to_heads``) are kept.
"""
import math

import os

import torch
import torch.nn as nn
import torch.nn.functional as F


class CaptureComplete(Exception):
    """Raised by a patched attention when its controller has every map it needs.

    The reference discards the UNet output of a capture pass
    (``ptp_utils.py:246-252``), and nothing after the 4th captured layer feeds the
    loss, so the forward may stop there (SURVEY.md §7 "UNet early exit").
    """


# --------------------------------------------------------------------------- libskp UNet-side kernels
# GroupNorm(+SiLU) with folded conv bias / time embedding, residual + bias, and the attention's
# fused softmax backward run on libskp when True (HIP tensors, frozen parameters); False is the
# plain-torch model (the tests compare the two).
USE_FUSED_GROUPNORM = True
USE_SKP_LAYERNORM = True   # tests switch it: False = ATen LayerNorm


def _fused(x, *modules):
    """The libskp UNet-side kernels apply: HIP tensor, frozen parameters."""
    return USE_FUSED_GROUPNORM and x.is_cuda and not any(p.requires_grad for m in modules for p in m.parameters())


def _conv_in(conv, x):
    """An input 3×3 convolution (latent or RGB channels): Winograd (channels zero-padded to a
    multiple of 4) when the fused kernels apply."""
    if _fused(x, conv):
        from .. import ops
        return ops.conv3x3(x, conv.weight, conv.bias)
    return conv(x)


def _ln(norm, x):
    """nn.LayerNorm ``norm`` on x: the libskp kernel on the HIP device (frozen affine
    parameters), elsewhere plain torch."""
    if USE_SKP_LAYERNORM and _fused(x, norm):
        from .. import ops
        return ops.layer_norm(x, norm.weight, norm.bias, norm.eps)
    return norm(x)


# A/B switch: 0 = the residual consumers of a norm's input get their gradient summed by autograd
NORM_RES = True


def _ln_res(norm, x):
    """(norm(x), x): on the fused path the second output hands x to the residual add, whose
    gradient the LayerNorm backward kernel then adds in its own pass (ops.layer_norm_res)."""
    if NORM_RES and USE_SKP_LAYERNORM and _fused(x, norm) and torch.is_grad_enabled() and x.requires_grad:
        from .. import ops
        return ops.layer_norm_res(x, norm.weight, norm.bias, norm.eps)
    return _ln(norm, x), x


def gn_act_res(norm, x, act):
    """(act(norm(x)), x) with the second output for x's other consumer (residual / shortcut): its
    gradient joins the GroupNorm backward kernel (ops.group_norm_act_res) on the fused path."""
    if NORM_RES and _fused(x, norm) and torch.is_grad_enabled() and x.requires_grad:
        from .. import ops
        return ops.group_norm_act_res(x, norm.weight, norm.bias, norm.num_groups, norm.eps, act)
    return gn_act(norm, x, act), x


def gn_act(norm, x, act, shift=None):
    """act(norm(x + shift)) for an nn.GroupNorm ``norm`` (``shift``: None or a per-(sample,
    channel) offset (B or 1, C)): on the HIP device the fused libskp kernel (frozen affine
    parameters, input gradient only, shift folded into its loads); elsewhere plain torch."""
    if _fused(x, norm):
        from .. import ops
        return ops.group_norm_act(x, norm.weight, norm.bias, norm.num_groups, norm.eps, act, shift)
    if shift is not None:
        x = x + shift.reshape(-1, x.shape[1], 1, 1)
    y = norm(x)
    return F.silu(y) if act else y


# --------------------------------------------------------------------------- attention
class CrossAttention(nn.Module):
    """diffusers-0.8.0 ``CrossAttention`` (bias-free q/k/v, ``to_out=[Linear, Dropout]``)."""

    # "math" is the literal GEMM + softmax form of diffusers 0.8.0 (fastest fp32 path on
    # MI355X, measured); "sdpa" routes the un-captured attention through torch SDPA.
    backend = "math"

    def __init__(self, query_dim, cross_attention_dim=None, heads=8, dim_head=64, dropout=0.0, bias=False):
        super().__init__()
        inner_dim = dim_head * heads
        cross_attention_dim = cross_attention_dim if cross_attention_dim is not None else query_dim
        self.scale = dim_head ** -0.5
        self.heads = heads
        self.to_q = nn.Linear(query_dim, inner_dim, bias=bias)
        self.to_k = nn.Linear(cross_attention_dim, inner_dim, bias=bias)
        self.to_v = nn.Linear(cross_attention_dim, inner_dim, bias=bias)
        self.to_out = nn.ModuleList([nn.Linear(inner_dim, query_dim), nn.Dropout(dropout)])

    def reshape_heads_to_batch_dim(self, tensor):
        b, s, dim = tensor.shape
        h = self.heads
        return tensor.reshape(b, s, h, dim // h).permute(0, 2, 1, 3).reshape(b * h, s, dim // h)

    def reshape_batch_dim_to_heads(self, tensor):
        bh, s, d = tensor.shape
        h = self.heads
        return tensor.reshape(bh // h, h, s, d).permute(0, 2, 1, 3).reshape(bh // h, s, d * h)

    def forward(self, x, context=None, mask=None):
        context = x if context is None else context
        if mask is None and USE_FUSED_GROUPNORM and x.is_cuda and CrossAttention.backend == "math":
            from .. import ops   # attention straight on the (B, S, H·d) projections: no head permutes
            one = None
            if context is x and ops.QKV_FUSED and _fused(x, self.to_q, self.to_k, self.to_v) and \
                    self.to_q.bias is None and self.to_k.bias is None and self.to_v.bias is None:
                # self-attention: q, k, v in one GEMM, their input gradients summed inside it
                qf, kf, vf = ops.qkv_projection(x, self.to_q.weight, self.to_k.weight, self.to_v.weight)
            else:
                qf = self.to_q(x)
                one = _shared_context(context)
                if one is not None:   # one sequence for the whole batch: projected once
                    k1, v1 = shared_kv(self, one)
                    kf, vf = k1.expand(x.shape[0], -1, -1), v1.expand(x.shape[0], -1, -1)
                else:
                    kf, vf = kv_projection(self, context)
            out = ops.attention_heads(qf, kf, vf, self.heads, self.scale)
            if out is None and one is not None and SHARED_HEAD_MAJOR and torch.is_grad_enabled():
                out = shared_context_attention(qf, k1, v1, self.heads, self.scale)
            if out is not None:
                return self.to_out[1](self.to_out[0](out))
            q = self.reshape_heads_to_batch_dim(qf)
            k, v = kf, vf
        else:
            q = self.reshape_heads_to_batch_dim(self.to_q(x))
            k, v = kv_projection(self, context)
        k = self.reshape_heads_to_batch_dim(k)
        v = self.reshape_heads_to_batch_dim(v)
        out = attention_core(q, k, v, self.scale, mask, self.heads)
        out = self.reshape_batch_dim_to_heads(out)
        return self.to_out[1](self.to_out[0](out))


SHARED_KV = True
# A/B switch: 0 = a batch-shared context's k / v are expanded to the batch and head-permuted with it
SHARED_HEAD_MAJOR = True


def _shared_context(context):
    """The one (1, L, C) sequence of a context whose batch is a stride-0 expansion (the token
    embedding every image of a batched pass shares), else None.  When the expansion is a view of
    that sequence (``ctx.expand(B, -1, -1)``, ptp_utils.find_pred_noise) the sequence itself is
    returned, so every layer's gradient lands on it directly: slicing the expansion (``[:1]``)
    makes autograd build a zero-filled (B, L, C) gradient per layer and sum those across layers."""
    if SHARED_KV and context.dim() == 3 and context.shape[0] > 1 and context.stride(0) == 0:
        base = context._base
        if (base is not None and base.dim() == 3 and base.shape[0] == 1 and base.shape[1:] == context.shape[1:]
                and base.stride()[1:] == context.stride()[1:] and base.data_ptr() == context.data_ptr()):
            return base
        return context[:1]
    return None


def shared_kv(attn, one):
    """to_k(one), to_v(one) of the (1, L, C) context the batch shares: one GEMM against [Wk; Wv]
    whose input gradient sums both projections' (ops.qkv_projection) on the fused path."""
    from .. import ops
    if ops.QKV_FUSED and _fused(one, attn.to_k, attn.to_v) and attn.to_k.bias is None and attn.to_v.bias is None:
        return ops.qkv_projection(one, attn.to_k.weight, attn.to_v.weight)
    return attn.to_k(one), attn.to_v(one)


def shared_context_attention(qf, k1, v1, H, scale):
    """softmax(q kᵀ·scale) v per head for (B, S, H·d) queries against ONE (1, L, H·d) key / value
    sequence shared by the batch, with the heads outermost: q as (H, B·S, d), k / v as (H, L, d),
    so each head is one GEMM over all B·S query rows (no per-image copy of the shared keys and
    values, and their gradients come out of the GEMMs already summed over the batch — no
    batch-expanded gradient and no reduction over it).  Same per-(query, head) arithmetic as the
    (B·H, S, d) form.  Returns (B, S, H·d)."""
    B, S, C = qf.shape
    L, d = k1.shape[1], C // H
    q = qf.reshape(B, S, H, d).permute(2, 0, 1, 3).reshape(H, B * S, d)
    k = k1.reshape(L, H, d).transpose(0, 1).contiguous()
    v = v1.reshape(L, H, d).transpose(0, 1).contiguous()
    o = attention_core(q, k, v, scale)
    return o.reshape(H, B, S, d).permute(1, 2, 0, 3).reshape(B, S, C)


def kv_projection(attn, context):
    """to_k(context), to_v(context).  A context whose batch is a stride-0 expansion of one
    sequence (the token embedding shared by every image of a batched pass) is projected once
    and the result expanded: the same values, 1/B of the GEMM work forward and backward."""
    one = _shared_context(context)
    if one is not None:
        B = context.shape[0]
        k1, v1 = shared_kv(attn, one)
        return k1.expand(B, -1, -1), v1.expand(B, -1, -1)
    return attn.to_k(context), attn.to_v(context)


def attention_core(q, k, v, scale, mask=None, heads=1):
    """softmax(q kᵀ · scale) v over (B·H, S, D) tensors (diffusers-0.8.0 semantics)."""
    if mask is None and CrossAttention.backend == "sdpa":
        return F.scaled_dot_product_attention(q.unsqueeze(0), k.unsqueeze(0), v.unsqueeze(0), scale=scale)[0]
    if mask is None and USE_FUSED_GROUPNORM and q.is_cuda and torch.is_grad_enabled() and \
            (q.requires_grad or k.requires_grad or v.requires_grad):
        from .. import ops   # same forward; one fused pass for the softmax backward
        return ops.math_attention(q, k, v, scale)
    if mask is None and USE_FUSED_GROUPNORM and q.is_cuda:
        from .. import ops   # no gradient needed: fused online-softmax attention / in-place softmax
        return ops.attention_nograd(q, k, v, scale)
    sim = torch.baddbmm(torch.empty(q.shape[0], q.shape[1], k.shape[1], dtype=q.dtype, device=q.device),
                        q, k.transpose(1, 2), beta=0, alpha=scale)
    if mask is not None:
        b = mask.shape[0]
        m = mask.reshape(b, -1)[:, None, :].repeat(heads, 1, 1)
        sim = sim.masked_fill(~m, -torch.finfo(sim.dtype).max)
    return torch.bmm(sim.softmax(dim=-1), v)


class GEGLU(nn.Module):
    def __init__(self, dim_in, dim_out):
        super().__init__()
        self.proj = nn.Linear(dim_in, dim_out * 2)

    def forward(self, x):
        h = self.proj(x)
        if USE_FUSED_GROUPNORM and h.is_cuda:
            from .. import ops   # one fused pass each way (skp_geglu_fwd / _bwd)
            return ops.geglu(h)
        x, gate = h.chunk(2, dim=-1)
        return x * F.gelu(gate)


class FeedForward(nn.Module):
    def __init__(self, dim, mult=4, dropout=0.0):
        super().__init__()
        inner = dim * mult
        self.net = nn.ModuleList([GEGLU(dim, inner), nn.Dropout(dropout), nn.Linear(inner, dim)])

    def forward(self, x):
        for m in self.net:
            x = m(x)
        return x


class BasicTransformerBlock(nn.Module):
    def __init__(self, dim, n_heads, d_head, cross_attention_dim):
        super().__init__()
        self.attn1 = CrossAttention(dim, heads=n_heads, dim_head=d_head)
        self.ff = FeedForward(dim)
        self.attn2 = CrossAttention(dim, cross_attention_dim=cross_attention_dim, heads=n_heads, dim_head=d_head)
        self.norm1 = nn.LayerNorm(dim)
        self.norm2 = nn.LayerNorm(dim)
        self.norm3 = nn.LayerNorm(dim)

    def forward(self, h, context=None):
        y, h = _ln_res(self.norm1, h)
        h = self.attn1(y) + h
        y, h = _ln_res(self.norm2, h)
        h = self.attn2(y, context=context) + h
        y, h = _ln_res(self.norm3, h)
        return self.ff(y) + h


class Transformer2DModel(nn.Module):
    """Spatial transformer: SD-1.x (conv proj_in/proj_out, one BasicTransformerBlock) or, with
    ``linear_proj`` and ``depth`` > 1, SDXL's (Linear projections on the (B, HW, C) tokens,
    ``depth`` BasicTransformerBlocks)."""

    def __init__(self, num_attention_heads, attention_head_dim, in_channels, cross_attention_dim, norm_num_groups=32,
                 depth=1, linear_proj=False):
        super().__init__()
        inner = num_attention_heads * attention_head_dim
        self.linear_proj = linear_proj
        self.norm = nn.GroupNorm(norm_num_groups, in_channels, eps=1e-6, affine=True)
        self.proj_in = nn.Linear(in_channels, inner) if linear_proj else nn.Conv2d(in_channels, inner, 1)
        self.transformer_blocks = nn.ModuleList(
            [BasicTransformerBlock(inner, num_attention_heads, attention_head_dim, cross_attention_dim)
             for _ in range(depth)])
        self.proj_out = nn.Linear(inner, in_channels) if linear_proj else nn.Conv2d(inner, in_channels, 1)

    def forward(self, x, encoder_hidden_states=None):
        b, c, hh, ww = x.shape
        x, res = gn_act_res(self.norm, x, False)
        if not self.linear_proj and _fused(x, self.proj_in, self.proj_out):
            # 1×1 projections as strided batched GEMMs straight between NCHW and (B, HW, C')
            from .. import ops
            x = ops.tokens_proj_in(x, self.proj_in.weight, self.proj_in.bias)
            for blk in self.transformer_blocks:
                x = blk(x, context=encoder_hidden_states)
            return ops.tokens_proj_out(x, self.proj_out.weight, self.proj_out.bias, res)
        if self.linear_proj:
            x = self.proj_in(x.permute(0, 2, 3, 1).reshape(b, hh * ww, c))
        else:
            x = self.proj_in(x)
            x = x.permute(0, 2, 3, 1).reshape(b, hh * ww, x.shape[1])
        inner = x.shape[-1]
        for blk in self.transformer_blocks:
            x = blk(x, context=encoder_hidden_states)
        if self.linear_proj:
            return self.proj_out(x).reshape(b, hh, ww, c).permute(0, 3, 1, 2) + res
        x = x.reshape(b, hh, ww, inner).permute(0, 3, 1, 2)
        return self.proj_out(x) + res


# --------------------------------------------------------------------------- resnets
class ResnetBlock2D(nn.Module):
    def __init__(self, in_channels, out_channels=None, temb_channels=1280, groups=32, eps=1e-5):
        super().__init__()
        out_channels = in_channels if out_channels is None else out_channels
        self.norm1 = nn.GroupNorm(groups, in_channels, eps=eps, affine=True)
        self.conv1 = nn.Conv2d(in_channels, out_channels, 3, 1, 1)
        self.time_emb_proj = nn.Linear(temb_channels, out_channels) if temb_channels is not None else None
        self.norm2 = nn.GroupNorm(groups, out_channels, eps=eps, affine=True)
        self.dropout = nn.Dropout(0.0)
        self.conv2 = nn.Conv2d(out_channels, out_channels, 3, 1, 1)
        self.conv_shortcut = nn.Conv2d(in_channels, out_channels, 1) if in_channels != out_channels else None

    def forward(self, x, temb=None):
        if _fused(x, self.conv1, self.conv2, self.norm2):
            # conv1's bias and the time embedding enter norm2 as its input shift, conv2's bias
            # the residual add: neither is a separate pass over the activations
            # (3×3 convolutions: Winograd F(4×4, 3×3) where the shape fills the chip, else MIOpen)
            from .. import ops
            y, x = gn_act_res(self.norm1, x, True)   # x goes on to the residual / shortcut
            h = ops.conv3x3(y, self.conv1.weight)
            shift = self.conv1.bias[None]
            if temb is not None and self.time_emb_proj is not None:
                shift = shift + self.time_emb_proj(F.silu(temb))
            bias = self.conv2.bias
            if self.conv_shortcut is not None:
                if _fused(x, self.conv_shortcut):
                    # the shortcut as one batched GEMM on NCHW; its bias joins conv2's in the epilogue
                    x = ops.conv1x1(x, self.conv_shortcut.weight)
                    bias = bias + self.conv_shortcut.bias
                else:
                    x = self.conv_shortcut(x)
            return ops.conv3x3(self.dropout(gn_act(self.norm2, h, True, shift)), self.conv2.weight, bias, x)
        h = self.conv1(gn_act(self.norm1, x, True))
        if temb is not None and self.time_emb_proj is not None:
            h = h + self.time_emb_proj(F.silu(temb))[:, :, None, None]
        h = self.conv2(self.dropout(gn_act(self.norm2, h, True)))
        if self.conv_shortcut is not None:
            x = self.conv_shortcut(x)
        return x + h


class Downsample2D(nn.Module):
    def __init__(self, channels, padding=1):
        super().__init__()
        self.padding = padding
        self.conv = nn.Conv2d(channels, channels, 3, stride=2, padding=padding)

    def forward(self, x):
        if self.padding == 0 and _fused(x, self.conv):
            from .. import ops
            if ops.conv3x3_s2_eligible(x, self.conv.weight):   # no padded copy, no MIOpen glue
                return ops.conv3x3_s2(x, self.conv.weight, self.conv.bias)
        if self.padding == 0:
            # F.pad(x, (0, 1, 0, 1)) without F.pad's zero fill of the whole output (the VAE's
            # 512² / 256² levels: a 1 GB fill per step): copy x, zero only the new row and column
            B, C, H, W = x.shape
            xp = x.new_empty(B, C, H + 1, W + 1)
            xp[:, :, :H, :W] = x
            xp[:, :, H, :].zero_()
            xp[:, :, :H, W].zero_()
            x = xp
        return self.conv(x)


class Upsample2D(nn.Module):
    def __init__(self, channels):
        super().__init__()
        self.conv = nn.Conv2d(channels, channels, 3, padding=1)

    def forward(self, x, output_size=None):
        if output_size is None:
            x = F.interpolate(x, scale_factor=2.0, mode="nearest")
        else:
            x = F.interpolate(x, size=output_size, mode="nearest")
        if _fused(x, self.conv):
            from .. import ops
            return ops.conv3x3(x, self.conv.weight, self.conv.bias)
        return self.conv(x)


# --------------------------------------------------------------------------- blocks
class CrossAttnDownBlock2D(nn.Module):
    def __init__(self, in_ch, out_ch, temb, heads, ctx_dim, add_downsample, groups=32, depth=1, linear_proj=False):
        super().__init__()
        self.resnets = nn.ModuleList([ResnetBlock2D(in_ch if i == 0 else out_ch, out_ch, temb, groups) for i in range(2)])
        self.attentions = nn.ModuleList([Transformer2DModel(heads, out_ch // heads, out_ch, ctx_dim, groups, depth,
                                                            linear_proj) for _ in range(2)])
        self.downsamplers = nn.ModuleList([Downsample2D(out_ch)]) if add_downsample else None

    def forward(self, h, temb, context):
        outs = ()
        for resnet, attn in zip(self.resnets, self.attentions):
            h = attn(resnet(h, temb), encoder_hidden_states=context)
            outs += (h,)
        if self.downsamplers is not None:
            h = self.downsamplers[0](h)
            outs += (h,)
        return h, outs


class DownBlock2D(nn.Module):
    def __init__(self, in_ch, out_ch, temb, add_downsample, groups=32):
        super().__init__()
        self.resnets = nn.ModuleList([ResnetBlock2D(in_ch if i == 0 else out_ch, out_ch, temb, groups) for i in range(2)])
        self.downsamplers = nn.ModuleList([Downsample2D(out_ch)]) if add_downsample else None

    def forward(self, h, temb, context=None):
        outs = ()
        for resnet in self.resnets:
            h = resnet(h, temb)
            outs += (h,)
        if self.downsamplers is not None:
            h = self.downsamplers[0](h)
            outs += (h,)
        return h, outs


class _UpBase(nn.Module):
    def _make_resnets(self, in_ch, out_ch, prev_ch, temb, groups=32):
        res = []
        for i in range(3):
            skip = in_ch if i == 2 else out_ch
            rin = prev_ch if i == 0 else out_ch
            res.append(ResnetBlock2D(rin + skip, out_ch, temb, groups))
        return nn.ModuleList(res)


class CrossAttnUpBlock2D(_UpBase):
    def __init__(self, in_ch, out_ch, prev_ch, temb, heads, ctx_dim, add_upsample, groups=32, depth=1,
                 linear_proj=False):
        super().__init__()
        self.resnets = self._make_resnets(in_ch, out_ch, prev_ch, temb, groups)
        self.attentions = nn.ModuleList([Transformer2DModel(heads, out_ch // heads, out_ch, ctx_dim, groups, depth,
                                                            linear_proj) for _ in range(3)])
        self.upsamplers = nn.ModuleList([Upsample2D(out_ch)]) if add_upsample else None

    def forward(self, h, res_tuple, temb, context, upsample_size=None):
        for resnet, attn in zip(self.resnets, self.attentions):
            skip = res_tuple[-1]
            res_tuple = res_tuple[:-1]
            h = torch.cat([h, skip], dim=1)
            h = attn(resnet(h, temb), encoder_hidden_states=context)
        if self.upsamplers is not None:
            h = self.upsamplers[0](h, upsample_size)
        return h


class UpBlock2D(_UpBase):
    def __init__(self, in_ch, out_ch, prev_ch, temb, add_upsample, groups=32):
        super().__init__()
        self.resnets = self._make_resnets(in_ch, out_ch, prev_ch, temb, groups)
        self.upsamplers = nn.ModuleList([Upsample2D(out_ch)]) if add_upsample else None

    def forward(self, h, res_tuple, temb, context=None, upsample_size=None):
        for resnet in self.resnets:
            skip = res_tuple[-1]
            res_tuple = res_tuple[:-1]
            h = resnet(torch.cat([h, skip], dim=1), temb)
        if self.upsamplers is not None:
            h = self.upsamplers[0](h, upsample_size)
        return h


class UNetMidBlock2DCrossAttn(nn.Module):
    def __init__(self, ch, temb, heads, ctx_dim, groups=32, depth=1, linear_proj=False):
        super().__init__()
        self.resnets = nn.ModuleList([ResnetBlock2D(ch, ch, temb, groups) for _ in range(2)])
        self.attentions = nn.ModuleList([Transformer2DModel(heads, ch // heads, ch, ctx_dim, groups, depth,
                                                            linear_proj)])

    def forward(self, h, temb, context):
        h = self.resnets[0](h, temb)
        h = self.attentions[0](h, encoder_hidden_states=context)
        return self.resnets[1](h, temb)


class TimestepEmbedding(nn.Module):
    def __init__(self, ch, dim):
        super().__init__()
        self.linear_1 = nn.Linear(ch, dim)
        self.linear_2 = nn.Linear(dim, dim)

    def forward(self, x):
        return self.linear_2(F.silu(self.linear_1(x)))


def timestep_embedding(timesteps, dim, flip_sin_to_cos=True, downscale_freq_shift=0.0, max_period=10000):
    half = dim // 2
    exponent = -math.log(max_period) * torch.arange(half, dtype=torch.float32, device=timesteps.device)
    exponent = exponent / (half - downscale_freq_shift)
    emb = timesteps[:, None].float() * torch.exp(exponent)[None, :]
    emb = torch.cat([torch.sin(emb), torch.cos(emb)], dim=-1)
    if flip_sin_to_cos:
        emb = torch.cat([emb[:, half:], emb[:, :half]], dim=-1)
    return emb


class UNet2DConditionModel(nn.Module):
    """SD-1.5 UNet: blocks (320, 640, 1280, 1280), 8 heads, cross-attention dim 768."""

    def __init__(self, in_channels=4, out_channels=4, block_out_channels=(320, 640, 1280, 1280),
                 cross_attention_dim=768, attention_head_dim=8, norm_num_groups=32):
        super().__init__()
        self.cross_attention_dim = cross_attention_dim
        ch0 = block_out_channels[0]
        temb = ch0 * 4
        heads = attention_head_dim
        self.conv_in = nn.Conv2d(in_channels, ch0, 3, padding=1)
        self.time_embedding = TimestepEmbedding(ch0, temb)
        self.down_blocks = nn.ModuleList()
        out_ch = ch0
        for i in range(4):
            in_ch, out_ch = out_ch, block_out_channels[i]
            last = i == 3
            if i < 3:
                self.down_blocks.append(CrossAttnDownBlock2D(in_ch, out_ch, temb, heads, cross_attention_dim, not last,
                                                             norm_num_groups))
            else:
                self.down_blocks.append(DownBlock2D(in_ch, out_ch, temb, not last, norm_num_groups))
        self.mid_block = UNetMidBlock2DCrossAttn(block_out_channels[-1], temb, heads, cross_attention_dim,
                                                 norm_num_groups)
        self.up_blocks = nn.ModuleList()
        rev = list(reversed(block_out_channels))
        out_ch = rev[0]
        for i in range(4):
            prev_ch, out_ch = out_ch, rev[i]
            in_ch = rev[min(i + 1, 3)]
            last = i == 3
            if i == 0:
                self.up_blocks.append(UpBlock2D(in_ch, out_ch, prev_ch, temb, not last, norm_num_groups))
            else:
                self.up_blocks.append(CrossAttnUpBlock2D(in_ch, out_ch, prev_ch, temb, heads, cross_attention_dim,
                                                         not last, norm_num_groups))
        self.conv_norm_out = nn.GroupNorm(norm_num_groups, ch0, eps=1e-5)
        self.conv_act = nn.SiLU()
        self.conv_out = nn.Conv2d(ch0, out_channels, 3, padding=1)
        self.time_proj_dim = ch0

    def forward(self, sample, timestep, encoder_hidden_states, return_dict=True):
        if not torch.is_tensor(timestep):
            timestep = torch.tensor([timestep], dtype=torch.long, device=sample.device)
        timesteps = timestep.reshape(-1).to(sample.device).expand(sample.shape[0])
        emb = self.time_embedding(timestep_embedding(timesteps, self.time_proj_dim).to(sample.dtype))
        h = _conv_in(self.conv_in, sample)
        res = (h,)
        for blk in self.down_blocks:
            h, r = blk(h, emb, encoder_hidden_states)
            res += r
        h = self.mid_block(h, emb, encoder_hidden_states)
        for i, blk in enumerate(self.up_blocks):
            n = len(blk.resnets)
            r, res = res[-n:], res[:-n]
            size = res[-1].shape[2:] if (i < 3) else None
            h = blk(h, r, emb, encoder_hidden_states, upsample_size=size)
        h = self.conv_out(gn_act(self.conv_norm_out, h, True))
        return {"sample": h} if return_dict else (h,)
