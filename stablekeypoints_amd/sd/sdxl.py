"""SDXL UNet (diffusers UNet2DConditionModel at the stable-diffusion-xl-base-1.0 config), fp32.

SURVEY.md §8 A16 (config 5): the reference's SDXL monkey-patch (``sdxl_monkey_patch.py``) is
inert, so the build defines SDXL capture as A1–A12 at SDXL shapes.  This module supplies the
model those shapes come from; the capture hook, stores and kernels are the SD-1.5 ones:

- blocks (320, 640, 1280) with 2 resnets per down block and 3 per up block; no attention at
  the highest resolution; transformer depths (1·2, 2·10) down, 10 mid, (10, 2) up;
- head dim 64 (10 heads at 640 channels, 20 at 1280), cross-attention width 2048, linear
  proj_in / proj_out;
- the "text_time" added conditioning: sinusoidal(256) of six time ids + a pooled text
  embedding (1280) → 2816 → MLP → added to the time embedding.  Without a text encoder the
  defaults are a zero pooled embedding and the time ids (H, W, 0, 0, H, W) of the input size.

With 1024² images the latents are 128²; the up_blocks[0] cross-attention runs at 32²
(S = 1024 ≤ the capture limit), 20 heads × 64: the A16 capture shape.
"""
import torch
import torch.nn as nn

from .unet import (_conv_in, CrossAttnDownBlock2D, CrossAttnUpBlock2D, DownBlock2D, TimestepEmbedding, UNetMidBlock2DCrossAttn,
                   UpBlock2D, gn_act, timestep_embedding)

SDXL_CONFIG = dict(block_out_channels=(320, 640, 1280), transformer_depth=(0, 2, 10), head_dim=64,
                   cross_attention_dim=2048, addition_time_embed_dim=256, pooled_dim=1280, norm_num_groups=32)


class SDXLUNet(nn.Module):
    def __init__(self, in_channels=4, out_channels=4, block_out_channels=(320, 640, 1280), transformer_depth=(0, 2, 10),
                 head_dim=64, cross_attention_dim=2048, addition_time_embed_dim=256, pooled_dim=1280,
                 norm_num_groups=32):
        super().__init__()
        self.cross_attention_dim = cross_attention_dim
        self.pooled_dim = pooled_dim
        self.addition_time_embed_dim = addition_time_embed_dim
        ch0 = block_out_channels[0]
        temb = ch0 * 4
        g = norm_num_groups
        n = len(block_out_channels)
        self.conv_in = nn.Conv2d(in_channels, ch0, 3, padding=1)
        self.time_embedding = TimestepEmbedding(ch0, temb)
        self.add_embedding = TimestepEmbedding(pooled_dim + 6 * addition_time_embed_dim, temb)
        self.time_proj_dim = ch0
        self.down_blocks = nn.ModuleList()
        out_ch = ch0
        for i in range(n):
            in_ch, out_ch = out_ch, block_out_channels[i]
            down = i < n - 1
            if transformer_depth[i] == 0:
                self.down_blocks.append(DownBlock2D(in_ch, out_ch, temb, down, g))
            else:
                self.down_blocks.append(CrossAttnDownBlock2D(in_ch, out_ch, temb, out_ch // head_dim,
                                                             cross_attention_dim, down, g, transformer_depth[i], True))
        top = block_out_channels[-1]
        self.mid_block = UNetMidBlock2DCrossAttn(top, temb, top // head_dim, cross_attention_dim, g,
                                                 transformer_depth[-1], True)
        self.up_blocks = nn.ModuleList()
        rev = list(reversed(block_out_channels))
        rdepth = list(reversed(transformer_depth))
        out_ch = rev[0]
        for i in range(n):
            prev_ch, out_ch = out_ch, rev[i]
            in_ch = rev[min(i + 1, n - 1)]
            up = i < n - 1
            if rdepth[i] == 0:
                self.up_blocks.append(UpBlock2D(in_ch, out_ch, prev_ch, temb, up, g))
            else:
                self.up_blocks.append(CrossAttnUpBlock2D(in_ch, out_ch, prev_ch, temb, out_ch // head_dim,
                                                         cross_attention_dim, up, g, rdepth[i], True))
        self.conv_norm_out = nn.GroupNorm(g, ch0, eps=1e-5)
        self.conv_out = nn.Conv2d(ch0, out_channels, 3, padding=1)

    def added_embedding(self, sample, added_cond_kwargs=None):
        b = sample.shape[0]
        kw = added_cond_kwargs or {}
        text = kw.get("text_embeds")
        if text is None:
            text = torch.zeros(b, self.pooled_dim, device=sample.device, dtype=sample.dtype)
        ids = kw.get("time_ids")
        if ids is None:
            h, w = sample.shape[2] * 8, sample.shape[3] * 8
            ids = torch.tensor([h, w, 0, 0, h, w], device=sample.device, dtype=sample.dtype).expand(b, 6)
        t = timestep_embedding(ids.reshape(-1), self.addition_time_embed_dim).reshape(b, -1).to(sample.dtype)
        return self.add_embedding(torch.cat([text.expand(b, -1), t], dim=-1))

    def forward(self, sample, timestep, encoder_hidden_states, return_dict=True, added_cond_kwargs=None):
        if not torch.is_tensor(timestep):
            timestep = torch.tensor([timestep], dtype=torch.long, device=sample.device)
        timesteps = timestep.reshape(-1).to(sample.device).expand(sample.shape[0])
        emb = self.time_embedding(timestep_embedding(timesteps, self.time_proj_dim).to(sample.dtype))
        emb = emb + self.added_embedding(sample, added_cond_kwargs)
        h = _conv_in(self.conv_in, sample)
        res = (h,)
        for blk in self.down_blocks:
            h, r = blk(h, emb, encoder_hidden_states)
            res += r
        h = self.mid_block(h, emb, encoder_hidden_states)
        for i, blk in enumerate(self.up_blocks):
            n = len(blk.resnets)
            r, res = res[-n:], res[:-n]
            size = res[-1].shape[2:] if res else None
            h = blk(h, r, emb, encoder_hidden_states, upsample_size=size)
        h = self.conv_out(gn_act(self.conv_norm_out, h, True))
        return {"sample": h} if return_dict else (h,)
