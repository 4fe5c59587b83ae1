"""The Z-Image-Turbo VAE decoder (diffusers AutoencoderKL with the FLUX.1 autoencoder config: 16 latent
channels, block widths 128/256/512/512, 2 + 1 ResnetBlocks per up block, GroupNorm(32) + SiLU,
a single-head attention in the mid block, nearest x2 upsampling + 3x3 conv; scaling 0.3611, shift
0.1159) in bf16, NHWC activations.

Reference: `ZImagePipeline` decodes `latents / scaling_factor + shift_factor` with its `vae`
(models/zImageTurbo.py:96-101).  Restated from the published config; no weights offline, parity with
diffusers UNPINNED.  Execution: the dense 3x3 convs whose widths fit run as libeggroll's implicit-GEMM
MFMA kernel (eggroll_conv_nhwc), conv_in / conv_out (16 / 3 channels) and the 1x1 shortcut on MIOpen /
hipBLASLt, GroupNorm + SiLU on eggroll_group_norm_nhwc (fp32 statistics), the mid-block attention on SDPA.
"""
from __future__ import annotations

import math
from typing import Sequence

import torch
import torch.nn.functional as F
from torch import nn

from . import kernels as K
from .dcae import conv_gemm_px, nchw, nhwc
from .lora import LoRALinear


def _p(*shape):
    return nn.Parameter(torch.empty(*shape, dtype=torch.bfloat16), requires_grad=False)


class GroupNorm(nn.Module):
    def __init__(self, c: int, groups: int = 32, eps: float = 1e-6):
        super().__init__()
        self.groups, self.eps = groups, eps
        self.weight, self.bias = _p(c), _p(c)
        self.use_kernel = True   # False: the fp32 torch form below (A/B, tests)

    def forward(self, x, silu: bool = True):  # NHWC bf16 -> NHWC bf16: GroupNorm (fp32 statistics) [+ SiLU]
        B, H, W, C = x.shape
        if self.use_kernel and x.is_cuda and C % 8 == 0 and C <= 2048:   # eggroll_group_norm_nhwc
            return K.group_norm_nhwc(x.contiguous(), self.groups, self.weight, self.bias, self.eps, silu)
        xf = x.float().view(B, H * W, self.groups, C // self.groups)
        var, mean = torch.var_mean(xf, dim=(1, 3), unbiased=False, keepdim=True)
        y = ((xf - mean) * torch.rsqrt(var + self.eps)).view(B, H, W, C) * self.weight.float() + self.bias.float()
        return (F.silu(y) if silu else y).to(torch.bfloat16)


class Conv(nn.Module):
    """ks x ks conv, pad ks // 2, NHWC in / out: libeggroll's implicit GEMM for 3x3 at supported widths."""

    def __init__(self, cin: int, cout: int, ks: int = 3):
        super().__init__()
        self.ks = ks
        self.weight = _p(cout, cin, ks, ks)
        self.bias = _p(cout)
        self.packed = None

    def forward(self, x):
        cin, cout = self.weight.shape[1], self.weight.shape[0]
        if self.ks == 3 and conv_gemm_px(cin) == 1 and cout % 64 == 0:
            key = (self.weight._version, self.weight.data_ptr())
            if self.packed is None or self.packed[0] != key:
                self.packed = (key, K.pack_conv3x3_weight(self.weight, 1))
            return K.conv3x3_nhwc(x.contiguous(), self.packed[1], self.bias, 1)
        if self.ks == 1:
            B, H, W, C = x.shape
            return F.linear(x.reshape(-1, C), self.weight.view(cout, cin), self.bias).view(B, H, W, cout)
        w = self.weight.contiguous(memory_format=torch.channels_last)
        y = F.conv2d(nchw(x.contiguous()), w, self.bias, padding=self.ks // 2)
        return nhwc(y).contiguous()


class ResnetBlock(nn.Module):
    def __init__(self, cin: int, cout: int):
        super().__init__()
        self.norm1, self.conv1 = GroupNorm(cin), Conv(cin, cout)
        self.norm2, self.conv2 = GroupNorm(cout), Conv(cout, cout)
        self.conv_shortcut = Conv(cin, cout, 1) if cin != cout else None

    def forward(self, x):
        h = self.conv2(self.norm2(self.conv1(self.norm1(x))))
        return h.add_(x if self.conv_shortcut is None else self.conv_shortcut(x))


class MidAttention(nn.Module):
    """diffusers Attention(c, heads=1, dim_head=c, norm=GroupNorm(32), residual) over the H*W tokens.
    to_q / to_k / to_v / to_out.0 are linears with diffusers' names (the Z-Image VAE-decoder LoRA targets,
    es_backend.py:598-608, unifed_es.py:492): with LoRA attached and a population context they run the
    population LoRA GEMM (kernel (2)); without LoRA, F.linear (hipBLASLt), as before."""

    def __init__(self, c: int):
        super().__init__()
        self.group_norm = GroupNorm(c)
        self.to_q, self.to_k, self.to_v = (LoRALinear(c, c, bias=True, lora=False) for _ in range(3))
        self.to_out = nn.ModuleList([LoRALinear(c, c, bias=True, lora=False)])
        for m in (self.to_q, self.to_k, self.to_v, self.to_out[0]):
            m.lib_small_m = 1 << 62   # no LoRA: the vendor GEMM (these ran as F.linear 1x1 convs)

    def forward(self, x):
        B, H, W, C = x.shape
        n = self.group_norm(x, silu=False).reshape(B, H * W, C)
        q, k, v = (m(n).view(B, 1, H * W, C) for m in (self.to_q, self.to_k, self.to_v))
        o = F.scaled_dot_product_attention(q, k, v, scale=C ** -0.5).view(B, H * W, C)
        return self.to_out[0](o).view(B, H, W, C).add_(x)


class FluxVAEDecoder(nn.Module):
    def __init__(self, latent_channels: int = 16, widths: Sequence[int] = (128, 256, 512, 512), layers: int = 2,
                 scaling_factor: float = 0.3611, shift_factor: float = 0.1159):
        super().__init__()
        self.scaling_factor, self.shift_factor = scaling_factor, shift_factor
        rev = list(reversed(widths))
        self.conv_in = Conv(latent_channels, rev[0])
        self.mid = nn.ModuleList([ResnetBlock(rev[0], rev[0]), MidAttention(rev[0]), ResnetBlock(rev[0], rev[0])])
        ups = []
        prev = rev[0]
        for i, c in enumerate(rev):
            blk = nn.Module()
            blk.resnets = nn.ModuleList([ResnetBlock(prev if j == 0 else c, c) for j in range(layers + 1)])
            blk.upsample = Conv(c, c) if i < len(rev) - 1 else None
            ups.append(blk)
            prev = c
        self.up_blocks = nn.ModuleList(ups)
        self.conv_norm_out = GroupNorm(widths[0])
        self.conv_out = Conv(widths[0], 3)

    @torch.no_grad()
    def init_weights(self, seed: int = 2):
        g = torch.Generator(device=self.conv_in.weight.device).manual_seed(seed)
        for name, p in self.named_parameters():
            if p.ndim >= 2:
                fan_in = p[0].numel()
                std = 1.0 / math.sqrt(fan_in)
                if name.endswith("conv2.weight") or name.endswith("to_out.0.weight"):
                    std *= 0.5
                p.copy_(torch.randn(p.shape, generator=g, device=p.device) * std)
            elif name.endswith("weight"):
                p.fill_(1.0)
            else:
                p.zero_()

    def forward(self, z):  # z [B, 16, h, w] (already z / scaling + shift) -> image [B, 3, 8h, 8w] in ~[-1, 1]
        x = self.conv_in(nhwc(z.to(torch.bfloat16)).contiguous())
        for m in self.mid:
            x = m(x)
        for blk in self.up_blocks:
            for r in blk.resnets:
                x = r(x)
            if blk.upsample is not None:
                x = blk.upsample(x.repeat_interleave(2, dim=1).repeat_interleave(2, dim=2))
        return nchw(self.conv_out(self.conv_norm_out(x)))
