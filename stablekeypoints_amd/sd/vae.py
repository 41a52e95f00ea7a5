"""SD-1.5 ``AutoencoderKL`` encoder half (diffusers-0.8.0 module names), plain PyTorch.

The hot path only encodes (reference ``ptp_utils.image2latent``,
``ptp_utils.py:289-304``: ``vae.encode(2x-1)["latent_dist"].mean * 0.18215``),
so the decoder is not built.  Sub-module names follow diffusers 0.8.0
(``encoder.*``, ``quant_conv``) so encoder weights of a real checkpoint load.
"""
import torch
import torch.nn as nn
import torch.nn.functional as F

from .unet import ResnetBlock2D, Downsample2D, gn_act, attention_core, _fused, _conv_in


class AttentionBlock(nn.Module):
    """diffusers-0.8.0 VAE ``AttentionBlock`` (one head, q/k/v/proj_attn Linear)."""

    def __init__(self, channels, norm_num_groups=32, eps=1e-6):
        super().__init__()
        self.channels = channels
        self.group_norm = nn.GroupNorm(norm_num_groups, channels, eps=eps, affine=True)
        self.query = nn.Linear(channels, channels)
        self.key = nn.Linear(channels, channels)
        self.value = nn.Linear(channels, channels)
        self.proj_attn = nn.Linear(channels, channels)

    def forward(self, x):
        b, c, h, w = x.shape
        res = x
        t = gn_act(self.group_norm, x, False).view(b, c, h * w).transpose(1, 2)
        q, k, v = self.query(t), self.key(t), self.value(t)
        o = attention_core(q, k, v, 1.0 / (c ** 0.5))
        o = self.proj_attn(o).transpose(1, 2).reshape(b, c, h, w)
        return o + res


class DownEncoderBlock2D(nn.Module):
    def __init__(self, in_ch, out_ch, add_downsample, groups=32):
        super().__init__()
        self.resnets = nn.ModuleList(
            [ResnetBlock2D(in_ch if i == 0 else out_ch, out_ch, temb_channels=None, groups=groups, eps=1e-6)
             for i in range(2)])
        self.downsamplers = nn.ModuleList([Downsample2D(out_ch, padding=0)]) if add_downsample else None

    def forward(self, x):
        for r in self.resnets:
            x = r(x)
        if self.downsamplers is not None:
            x = self.downsamplers[0](x)
        return x


class UNetMidBlock2D(nn.Module):
    def __init__(self, ch, groups=32):
        super().__init__()
        self.resnets = nn.ModuleList([ResnetBlock2D(ch, ch, temb_channels=None, groups=groups, eps=1e-6)
                                      for _ in range(2)])
        self.attentions = nn.ModuleList([AttentionBlock(ch, groups)])

    def forward(self, x):
        x = self.resnets[0](x)
        x = self.attentions[0](x)
        return self.resnets[1](x)


class Encoder(nn.Module):
    def __init__(self, in_channels=3, block_out_channels=(128, 256, 512, 512), latent_channels=4, norm_num_groups=32):
        super().__init__()
        g = norm_num_groups
        self.conv_in = nn.Conv2d(in_channels, block_out_channels[0], 3, padding=1)
        self.down_blocks = nn.ModuleList()
        out_ch = block_out_channels[0]
        for i, ch in enumerate(block_out_channels):
            in_ch, out_ch = out_ch, ch
            self.down_blocks.append(DownEncoderBlock2D(in_ch, out_ch, i < len(block_out_channels) - 1, g))
        self.mid_block = UNetMidBlock2D(block_out_channels[-1], g)
        self.conv_norm_out = nn.GroupNorm(g, block_out_channels[-1], eps=1e-6)
        self.conv_act = nn.SiLU()
        self.conv_out = nn.Conv2d(block_out_channels[-1], 2 * latent_channels, 3, padding=1)

    def forward(self, x):
        x = _conv_in(self.conv_in, x)
        for blk in self.down_blocks:
            x = blk(x)
        x = self.mid_block(x)
        return self.conv_out(gn_act(self.conv_norm_out, x, True))


class DiagonalGaussianDistribution:
    def __init__(self, parameters):
        self.mean, self.logvar = torch.chunk(parameters, 2, dim=1)


class AutoencoderKL(nn.Module):
    def __init__(self, latent_channels=4, block_out_channels=(128, 256, 512, 512), norm_num_groups=32):
        super().__init__()
        self.encoder = Encoder(block_out_channels=tuple(block_out_channels), latent_channels=latent_channels,
                               norm_num_groups=norm_num_groups)
        self.quant_conv = nn.Conv2d(2 * latent_channels, 2 * latent_channels, 1)

    def encode(self, x, return_dict=True):
        post = DiagonalGaussianDistribution(self.quant_conv(self.encoder(x)))
        return {"latent_dist": post} if return_dict else (post,)
