"""DC-AE f32c32 decoder (AutoencoderDC of Sana_Sprint_1.6B_1024px) in bf16, channels-last.

Reference: `AutoencoderDC.from_pretrained(model, subfolder="vae", torch_dtype=float32)` and
`vae.decode(pred_x0 / scaling_factor)` (models/SanaSprint.py:44-49, 157-160).  Restated from
the published dc-ae-f32c32-sana-1.0 architecture (decoder block widths 128/256/512/512/1024/1024,
3 layers per stage, ResBlocks at the three high-resolution stages and EfficientViT blocks with
ReLU multiscale linear attention at the three low-resolution stages, interpolate-upsampling with
pixel-shuffle shortcuts, RMSNorm).  No weights exist offline: parity with diffusers is UNPINNED;
shapes and FLOPs (~7.5 TFLOP per 1024^2 image) follow the architecture.  Runs on PyTorch-ROCm
(MIOpen convolutions) — it is not one of the libeggroll hot-path kernels.
"""
from __future__ import annotations

import math
from typing import Sequence

import torch
import torch.nn.functional as F
from torch import nn

CL = torch.channels_last


def _p(*shape, dtype=torch.bfloat16):
    return nn.Parameter(torch.empty(*shape, dtype=dtype), requires_grad=False)


class RMSNormC(nn.Module):
    """RMSNorm over channels of an NCHW (channels-last) tensor, with weight and bias."""

    def __init__(self, c: int, eps: float = 1e-5):
        super().__init__()
        self.eps = eps
        self.weight = _p(c)
        self.bias = _p(c)

    def forward(self, x):
        y = F.rms_norm(x.permute(0, 2, 3, 1), (x.shape[1],), self.weight, self.eps) + self.bias
        return y.permute(0, 3, 1, 2)


class Conv(nn.Module):
    def __init__(self, cin: int, cout: int, k: int, groups: int = 1, bias: bool = True):
        super().__init__()
        self.k, self.groups = k, groups
        self.weight = _p(cout, cin // groups, k, k)
        self.bias = _p(cout) if bias else None

    def forward(self, x):
        return F.conv2d(x, self.weight, self.bias, padding=self.k // 2, groups=self.groups)


class ResBlock(nn.Module):
    def __init__(self, c: int):
        super().__init__()
        self.conv1 = Conv(c, c, 3)
        self.conv2 = Conv(c, c, 3, bias=False)
        self.norm = RMSNormC(c)

    def forward(self, x):
        return self.norm(self.conv2(F.silu(self.conv1(x)))) + x


class GLUMBConvC(nn.Module):
    def __init__(self, c: int, expand: int = 4):
        super().__init__()
        h = c * expand
        self.conv_inverted = Conv(c, 2 * h, 1)
        self.conv_depth = Conv(2 * h, 2 * h, 3, groups=2 * h)
        self.conv_point = Conv(h, c, 1, bias=False)
        self.norm = RMSNormC(c)

    def forward(self, x):
        h = self.conv_depth(F.silu(self.conv_inverted(x)))
        a, g = h.chunk(2, dim=1)
        return self.norm(self.conv_point(a * F.silu(g))) + x


class MultiscaleLinearAttention(nn.Module):
    """SanaMultiscaleLinearAttention (kernel sizes (5,), head dim 32, ReLU linear attention)."""

    def __init__(self, c: int, head_dim: int = 32, scales: Sequence[int] = (5,)):
        super().__init__()
        self.heads = c // head_dim
        self.hd = head_dim
        inner = self.heads * head_dim
        self.to_q = _p(inner, c)
        self.to_k = _p(inner, c)
        self.to_v = _p(inner, c)
        self.ms_in = nn.ModuleList([Conv(3 * inner, 3 * inner, k, groups=3 * inner, bias=False) for k in scales])
        self.ms_out = nn.ModuleList([Conv(3 * inner, 3 * inner, 1, groups=3 * self.heads, bias=False) for _ in scales])
        self.to_out = _p(c, inner * (1 + len(scales)))
        self.norm_out = RMSNormC(c)

    def forward(self, x):
        B, C, H, W = x.shape
        t = x.permute(0, 2, 3, 1)                                               # [B,H,W,C]
        qkv = torch.cat([F.linear(t, self.to_q), F.linear(t, self.to_k), F.linear(t, self.to_v)], dim=-1)
        qkv = qkv.permute(0, 3, 1, 2)                                           # NCHW view, CL strides
        branches = [qkv] + [o(i(qkv)) for i, o in zip(self.ms_in, self.ms_out)]
        outs = []
        for br in branches:                                                     # [B, 3*inner, H, W]
            br = br.permute(0, 2, 3, 1).reshape(B, H * W, 3, self.heads, self.hd).float()
            q, k, v = F.relu(br[:, :, 0]), F.relu(br[:, :, 1]), br[:, :, 2]
            kv = torch.einsum("bnhj,bnhi->bhji", k, v)
            num = torch.einsum("bnhj,bhji->bnhi", q, kv)
            den = torch.einsum("bnhj,bhj->bnh", q, k.sum(1)).unsqueeze(-1)
            outs.append((num / (den + 1e-15)).reshape(B, H, W, -1).to(torch.bfloat16))
        y = F.linear(torch.cat(outs, dim=-1), self.to_out).permute(0, 3, 1, 2)
        return self.norm_out(y) + x


class EfficientViTBlock(nn.Module):
    def __init__(self, c: int):
        super().__init__()
        self.attn = MultiscaleLinearAttention(c)
        self.conv_out = GLUMBConvC(c)

    def forward(self, x):
        return self.conv_out(self.attn(x))


class UpBlock(nn.Module):
    """DCUpBlock2d(interpolate=True, shortcut=True): nearest x2 + 3x3 conv, + pixel-shuffle shortcut."""

    def __init__(self, cin: int, cout: int):
        super().__init__()
        self.conv = Conv(cin, cout, 3)
        self.repeats = cout * 4 // cin

    def forward(self, x):
        y = self.conv(F.interpolate(x, scale_factor=2, mode="nearest"))
        s = F.pixel_shuffle(x.repeat_interleave(self.repeats, dim=1), 2)
        return y + s


class DCAEDecoder(nn.Module):
    def __init__(self, latent_channels: int = 32, widths=(128, 256, 512, 512, 1024, 1024),
                 layers=(3, 3, 3, 3, 3, 3), vit_from: int = 3, scaling_factor: float = 0.41407):
        super().__init__()
        self.scaling_factor = scaling_factor
        self.latent_channels = latent_channels
        self.conv_in = Conv(latent_channels, widths[-1], 3)
        self.in_repeats = widths[-1] // latent_channels
        stages = []
        for i in reversed(range(len(widths))):
            blocks = []
            if i < len(widths) - 1:
                blocks.append(UpBlock(widths[i + 1], widths[i]))
            for _ in range(layers[i]):
                blocks.append(EfficientViTBlock(widths[i]) if i >= vit_from else ResBlock(widths[i]))
            stages.append(nn.Sequential(*blocks))
        self.stages = nn.ModuleList(stages)  # lowest resolution first
        self.norm_out = RMSNormC(widths[0])
        self.conv_out = Conv(widths[0], 3, 3)

    @torch.no_grad()
    def init_weights(self, seed: int = 1):
        g = torch.Generator(device=self.conv_in.weight.device).manual_seed(seed)
        for name, p in self.named_parameters():
            if p.ndim >= 2:
                std = 1.0 / math.sqrt(p[0].numel())
                p.copy_(torch.randn(p.shape, generator=g, device=p.device) * std * 0.5)
            elif name.endswith("weight"):
                p.fill_(1.0)
            else:
                p.zero_()

    def forward(self, z):  # z [B, 32, h, w] -> image [B, 3, 32h, 32w] in ~[-1, 1]
        z = z.to(torch.bfloat16).contiguous(memory_format=CL)
        x = self.conv_in(z) + z.repeat_interleave(self.in_repeats, dim=1)
        for st in self.stages:
            x = st(x)
        x = F.relu(self.norm_out(x))
        return self.conv_out(x)
