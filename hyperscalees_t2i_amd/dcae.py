"""DC-AE f32c32 decoder (AutoencoderDC of Sana_Sprint_1.6B_1024px) in bf16, NHWC activations.

Reference: `AutoencoderDC.from_pretrained(model, subfolder="vae", torch_dtype=float32)` and
`vae.decode(pred_x0 / scaling_factor)` (models/SanaSprint.py:44-49, 157-160).  Restated from
the published dc-ae-f32c32-sana-1.0 architecture (decoder block widths 128/256/512/512/1024/1024,
3 layers per stage, ResBlocks at the three high-resolution stages and EfficientViT blocks with
ReLU multiscale linear attention at the three low-resolution stages, interpolate-upsampling with
pixel-shuffle shortcuts, RMSNorm).  No weights exist offline: parity with diffusers is UNPINNED;
shapes and FLOPs (~7.5 TFLOP per 1024^2 image) follow the architecture.

Execution (not one of the ES hot-path kernels): activations stay NHWC
contiguous; the ResBlocks' dense 3x3 convs run as libeggroll's implicit-GEMM MFMA kernel
(eggroll_conv3x3_nhwc, conv1's bias + SiLU in its epilogue; conv2 + RMSNorm + residual in one launch), the remaining dense convs go to MIOpen
on channels-last views, 1x1 convs to hipBLASLt, and depthwise convs (+SiLU / GLU gate) to
libeggroll's eggroll_dwconv_nhwc.
"""
from __future__ import annotations

import math
from typing import Sequence

import torch
import torch.nn.functional as F
from torch import nn

from . import kernels as K
from . import lora


def _p(*shape, dtype=torch.bfloat16):
    return nn.Parameter(torch.empty(*shape, dtype=dtype), requires_grad=False)


def nchw(x):  # NHWC-contiguous -> NCHW view with channels-last strides (no copy)
    return x.permute(0, 3, 1, 2)


def nhwc(x):  # channels-last NCHW -> NHWC view (contiguous when x is channels-last)
    return x.permute(0, 2, 3, 1)


class RMSNormC(nn.Module):
    def __init__(self, c: int, eps: float = 1e-5):
        super().__init__()
        self.eps = eps
        self.weight = _p(c)
        self.bias = _p(c)

    def forward(self, x, res=None, act=None, shadow=None):  # NHWC; fused norm * w + b [act] [+ res]
        """An fp32 res is the fp32 residual stream: updated in place (res = norm(x) * w + b + res), shadow
        receiving its bf16 copy."""
        return K.rownorm(x.contiguous(), self.eps, layer=False, w=self.weight, b=self.bias, act=act, res=res,
                         shadow=shadow)


# conv_in on libeggroll's conv (channel-padded) instead of MIOpen: MIOpen's immediate-mode solver choice is
# made per process, and 8 ranks sharing one GPU produced S rows that differed from one process's for a
# timing-dependent subset of ranks (profiles/r13l_*); False restores F.conv2d (A/B)
LIB_SMALL_CIN = True


class Conv3x3(nn.Module):
    def __init__(self, cin: int, cout: int, bias: bool = True):
        super().__init__()
        self.weight = nn.Parameter(torch.empty(cout, cin, 3, 3, dtype=torch.bfloat16).contiguous(
            memory_format=torch.channels_last), requires_grad=False)
        self.bias = _p(cout) if bias else None

    def lib_small_cin(self, x) -> bool:
        """Input widths below libeggroll's 64-channel minimum (the decoder's conv_in, 32 latent channels): the
        input and weight zero-padded to 64 channels on the halo conv (exact: the pad terms are 0 * 0)."""
        cout, cin = self.weight.shape[0], self.weight.shape[1]
        return (LIB_SMALL_CIN and x.is_cuda and cin < 64 and 64 % cin == 0 and cout % 256 == 0 and cout <= 2048
                and x.shape[1] % 16 == 0 and x.shape[2] % 16 == 0)

    def forward(self, x):  # NHWC -> NHWC
        if self.lib_small_cin(x):
            key = (self.weight._version, self.weight.data_ptr())
            if getattr(self, "_pk_key", None) != key:
                w64 = F.pad(self.weight.detach(), (0, 0, 0, 0, 0, 64 - self.weight.shape[1]))
                self._pk, self._pk_key = K.pack_conv3x3_weight(w64, 1), key
            return K.conv3x3_nhwc(F.pad(x, (0, 64 - x.shape[-1])), self._pk, self.bias, 1)
        y = F.conv2d(nchw(x.contiguous()), self.weight, self.bias, padding=1)
        y = nhwc(y)
        return y if y.is_contiguous() else y.contiguous()


def conv_gemm_px(c: int) -> int:
    """Super-pixel width for libeggroll's implicit-GEMM 3x3 conv at c -> c channels (0: not eligible):
    1 for 128..2048 (c = 128 runs the 512 x 128 tile), 0 otherwise (MIOpen)."""
    if c < 128 or c > 2048 or c & (c - 1):
        return 0
    return 1


class ResBlock(nn.Module):
    """conv1 (+bias, SiLU) -> conv2 (no bias) -> RMSNorm + residual.  Both convs run as libeggroll's
    implicit-GEMM MFMA kernel (bias + SiLU fused into conv1's epilogue) when the width allows,
    else MIOpen + a bias/SiLU pass."""

    def __init__(self, c: int):
        super().__init__()
        self.conv1 = Conv3x3(c, c)
        self.conv2 = Conv3x3(c, c, bias=False)
        self.norm = RMSNormC(c)
        self.px = conv_gemm_px(c)
        self.packed = None

    def refresh_packed_weights(self):
        if self.px:
            self.packed = (K.pack_conv3x3_weight(self.conv1.weight, self.px),
                           self.conv1.bias.repeat(self.px).contiguous(),
                           K.pack_conv3x3_weight(self.conv2.weight, self.px))

    def forward(self, x):
        x = x.contiguous()
        if self.px and x.shape[2] % self.px == 0:
            if self.packed is None:
                self.refresh_packed_weights()
            w1, b1, w2 = self.packed
            h = K.conv3x3_nhwc(x, w1, b1, self.px, "silu")
            if w2.shape[0] in (128, 256):  # whole pixels per tile: RMSNorm + residual in conv2's epilogue
                n = self.norm
                return K.conv3x3_rmsnorm_nhwc(h, w2, None, self.px, n.eps, n.weight, n.bias, x)
            return self.norm(K.conv3x3_nhwc(h, w2, None, self.px), res=x)
        c1 = self.conv1
        h = nhwc(F.conv2d(nchw(x), c1.weight, None, padding=1)).contiguous()
        h = K.bias_act_(h, c1.bias, "silu")                       # bias + SiLU in one pass
        return self.norm(self.conv2(h), res=x)

    def forward_f32(self, x32, x16):
        """The block on the fp32 residual stream (x32 updated in place, x16 its bf16 shadow = the convs'
        input): conv1 + SiLU and conv2 on libeggroll's MFMA kernels (conv2 without the fused norm tail),
        then RMSNorm + the fp32 residual add in one row pass."""
        if self.px and x16.shape[2] % self.px == 0:
            if self.packed is None:
                self.refresh_packed_weights()
            w1, b1, w2 = self.packed
            h = K.conv3x3_nhwc(K.conv3x3_nhwc(x16, w1, b1, self.px, "silu"), w2, None, self.px)
        else:
            c1 = self.conv1
            h = nhwc(F.conv2d(nchw(x16), c1.weight, None, padding=1)).contiguous()
            h = self.conv2(K.bias_act_(h, c1.bias, "silu"))
        self.norm(h, res=x32, shadow=x16)
        return x32, x16

    def forward_reference(self, x):
        return self.norm(self.conv2(F.silu(self.conv1(x))), res=x)


class GLUMBConvC(nn.Module):
    """conv_inverted (1x1) -> SiLU -> dw3x3 -> GLU -> conv_point (1x1) -> RMSNorm, + residual."""

    def __init__(self, c: int, expand: int = 4):
        super().__init__()
        h = c * expand
        self.w_inv, self.b_inv = _p(2 * h, c), _p(2 * h)
        self.w_dw, self.b_dw = _p(9, 2 * h), _p(2 * h)      # [tap][C]
        self.w_point = _p(c, h)
        self.norm = RMSNormC(c)

    def forward(self, x, res32=None, shadow=None):  # NHWC
        """res32 (optional): the fp32 residual stream, updated in place instead of returning x + block(x)
        (shadow = its bf16 copy)."""
        B, H, W, C = x.shape
        if C <= 512:
            # 1x1 conv on the 8-phase GEMM, SiLU in the depthwise conv's staging (lora.SILU_IN_GEMM: in the
            # GEMM epilogue instead, the same bits; 3.5 % slower at 512 channels since round 5,
            # profiles/r09q_silu_placement.log).  At 1024 channels hipBLASLt's GEMM is faster.
            x2 = x.reshape(-1, C)
            if lora.FUSE_EPILOGUES and lora.SILU_IN_GEMM:
                h = K.lora_linear_pop_epi(x2, self.w_inv, self.b_inv, None, 0, 0, 0, 0.0, B * H * W, "silu")
                g = K.dwconv_nhwc(h.view(B, H, W, -1), self.w_dw, self.b_dw, 3, pre_silu=False, glu=True)
            else:
                h = K.lora_linear_pop(x2.contiguous(), self.w_inv, self.b_inv, None, 0, 0, 0, 0.0, B * H * W)
                g = K.dwconv_nhwc(h.view(B, H, W, -1), self.w_dw, self.b_dw, 3, pre_silu=True, glu=True)
        else:
            h = F.linear(x, self.w_inv, self.b_inv)
            g = K.dwconv_nhwc(h, self.w_dw, self.b_dw, 3, pre_silu=True, glu=True)
        return self.norm(F.linear(g, self.w_point), res=x if res32 is None else res32, shadow=shadow)


class MultiscaleLinearAttention(nn.Module):
    """SanaMultiscaleLinearAttention (kernel sizes (5,), head dim 32, ReLU linear attention)."""

    def __init__(self, c: int, head_dim: int = 32, scales: Sequence[int] = (5,)):
        super().__init__()
        self.heads, self.hd = c // head_dim, head_dim
        inner = self.heads * head_dim
        self.w_qkv = _p(3 * inner, c)                            # to_q | to_k | to_v (no bias)
        self.ms_dw = nn.ParameterList([_p(k * k, 3 * inner) for k in scales])   # depthwise, [tap][C]
        self.ms_pw = nn.ParameterList([_p(3 * self.heads, head_dim, head_dim) for _ in scales])  # grouped 1x1
        self.scales = list(scales)
        self.w_out = _p(c, inner * (1 + len(scales)))
        self.norm_out = RMSNormC(c)

    def _attend(self, br, out, planar=False):
        # br [B,H,W,3*inner]: per head group h, channels [q | k | v] of 32 each (the reference layout), or
        # planar [Q | K | V] with head h's q / k / v at column 32h of each plane
        B, H, W, C3 = br.shape
        flat = br.reshape(B * H * W, C3)
        inner = self.heads * self.hd
        if planar:
            K.linear_attention(flat, flat[:, inner:], flat[:, 2 * inner:], B, H * W, self.heads, self.hd,
                               relu_qk=True, out=out)
        else:
            K.linear_attention(flat, flat[:, self.hd:], flat[:, 2 * self.hd:], B, H * W, self.heads, 3 * self.hd,
                               relu_qk=True, out=out)

    # Planar q/k/v at the largest maps: the same channels, relabelled so that a head's q, k and v each
    # share 128-B lines with the neighbouring head's instead of with its own other two (whose bytes the
    # pass does not read): the linear attention at 8 x 128 x 128 x 16 heads 0.226 -> 0.186 ms; at 64^2
    # and below the reference layout is as fast (tools/la_probe.py).  w_qkv's rows, the depthwise
    # weights' channels and the grouped 1x1's 32-channel groups are permuted alike, so every branch
    # computes the same values in the permuted columns; the attention output layout is unchanged.
    PLANAR_MIN_TOKENS = 8192

    def _planar_weights(self):
        key = (self.w_qkv._version, self.w_qkv.data_ptr(),
               tuple((w._version, w.data_ptr()) for w in list(self.ms_dw) + list(self.ms_pw)))
        if getattr(self, "_planar_key", None) != key:
            hd, heads = self.hd, self.heads
            inner = heads * hd
            n = torch.arange(3 * inner, device=self.w_qkv.device)
            perm = (n % inner) // hd * (3 * hd) + n // inner * hd + n % hd   # planar column -> reference column
            gp = torch.arange(3 * heads, device=self.w_qkv.device)
            gperm = gp % heads * 3 + gp // heads                              # planar group -> reference group
            self._planar_w = (self.w_qkv[perm].contiguous(), [w[:, perm].contiguous() for w in self.ms_dw],
                              [w[gperm].contiguous() for w in self.ms_pw])
            self._planar_key = key
        return self._planar_w

    def forward(self, x, res32=None, shadow=None):  # NHWC; res32 / shadow: as GLUMBConvC.forward
        B, H, W, C = x.shape
        planar = H * W >= self.PLANAR_MIN_TOKENS
        w_qkv, ms_dw, ms_pw = self._planar_weights() if planar else (self.w_qkv, self.ms_dw, self.ms_pw)
        if C <= 512:   # K = 512: the 8-phase GEMM runs 955 vs hipBLASLt's 832-861 TF/s (r04_dcae_gemm_*.json)
            qkv = K.lora_linear_pop(x.reshape(-1, C), w_qkv, None, None, 0, 0, 0, 0.0, B * H * W).view(B, H, W, -1)
        else:          # K = 1024: hipBLASLt's stream-K GEMM is as fast or faster at these M
            qkv = F.linear(x, w_qkv)                              # [B,H,W,3*inner]
        inner = self.heads * self.hd
        # every branch's attention output lands in its column slice of one buffer (no concat pass)
        o = torch.empty((B * H * W, inner * (1 + len(self.scales))), dtype=x.dtype, device=x.device)
        self._attend(qkv, o[:, :inner], planar)
        for i, (ks, wdw, wpw) in enumerate(zip(self.scales, ms_dw, ms_pw)):
            # depthwise ks x ks + grouped 1x1 (G = 3h + {q,k,v} groups of 32, or their planar order) in one
            # kernel, output in the qkv layout, which the attention reads like the first branch
            pg = K.dwconv_pw_nhwc(qkv, wdw, wpw, ks).view(B * H * W, 3 * inner)
            self._attend(pg.view(B, H, W, 3 * inner), o[:, (i + 1) * inner:(i + 2) * inner], planar)
        y = F.linear(o.view(B, H, W, -1), self.w_out)
        return self.norm_out(y, res=x if res32 is None else res32, shadow=shadow)


class EfficientViTBlock(nn.Module):
    def __init__(self, c: int):
        super().__init__()
        self.attn = MultiscaleLinearAttention(c)
        self.conv_out = GLUMBConvC(c)

    def forward(self, x):
        return self.conv_out(self.attn(x))

    def forward_f32(self, x32, x16):
        self.attn(x16, res32=x32, shadow=x16)
        self.conv_out(x16, res32=x32, shadow=x16)
        return x32, x16


def subpixel_phase_weights(w3: torch.Tensor) -> torch.Tensor:
    """[Cout, Cin, 3, 3] kernel of conv3x3(nearest_up_x2(x)) -> [4*Cout, Cin, 2, 2] phase kernels of
    an equivalent pad-1 2x2 conv on x: phase (i, j) sums the 3x3 taps that land on the same
    low-resolution pixel (i=0: rows {0} | {1,2}; i=1: rows {0,1} | {2}; likewise columns)."""
    groups = {0: ([0], [1, 2]), 1: ([0, 1], [2])}
    out = []
    for i in (0, 1):
        for j in (0, 1):
            k = torch.zeros(w3.shape[0], w3.shape[1], 2, 2, dtype=torch.float32, device=w3.device)
            for a in (0, 1):
                for b in (0, 1):
                    k[:, :, a, b] = w3.float()[:, :, groups[i][a]][:, :, :, groups[j][b]].sum(dim=(2, 3))
            out.append(k)
    return torch.cat(out, dim=0)


# Up-block phase conv with the sub-pixel interleave + shortcut in its epilogue (one launch, no y4
# intermediate; eggroll_conv2x2_subpixel_nhwc, bitwise equal to the two-launch form, which False selects)
FUSED_SUBPIXEL = True


class UpBlock(nn.Module):
    """DCUpBlock2d(interpolate=True, shortcut=True): nearest x2 + 3x3 conv + pixel-shuffle shortcut.
    Executed as a pad-1 2x2 conv with 4*Cout sub-pixel phase outputs on the LOW-resolution input
    (4/9 of the FLOPs, no upsampled tensor) and one fused interleave + shortcut kernel; exact up to
    summation order (tests/test_gpu_kernels.py::test_subpixel_upblock_matches_reference)."""

    def __init__(self, cin: int, cout: int):
        super().__init__()
        self.conv = Conv3x3(cin, cout)           # the architecture's 3x3 weights (source of truth)
        self.repeats = cout * 4 // cin
        self.w4 = self.w4p = None

    def refresh_phase_weights(self):
        w4 = subpixel_phase_weights(self.conv.weight)
        self.w4 = w4.to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
        cin = self.w4.shape[1]
        # libeggroll's implicit-GEMM conv (ks 2) when the widths fit it, else MIOpen
        self.w4p = (K.pack_conv3x3_weight(self.w4, 1)
                    if 64 <= cin <= 2048 and cin & (cin - 1) == 0 and self.w4.shape[0] % 64 == 0 else None)

    def fused_ok(self) -> bool:
        """eggroll_conv2x2_subpixel_nhwc's shape rule (Cin a power of two in [64, 2048] — already required
        for w4p —, 4*Cout a multiple of 256 and <= 8192, 4*Cout / Cin in {1, 2, 4}); other widths take the
        two-launch conv + subpixel_shortcut form."""
        n4, cin = self.w4.shape[0], self.w4.shape[1]
        return (self.w4p is not None and FUSED_SUBPIXEL and n4 % 256 == 0 and n4 <= 8192 and n4 % cin == 0
                and n4 // cin in (1, 2, 4))

    def forward(self, x):  # NHWC
        if self.w4 is None:
            self.refresh_phase_weights()
        x = x.contiguous()
        if self.fused_ok():
            return K.conv2x2_subpixel(x, self.w4p, x, bias=self.conv.bias)   # one launch, the same bits
        # bias-free phase conv; the conv bias is added in fp32 by the interleave kernel
        if self.w4p is not None:
            y4 = K.conv_nhwc(x, self.w4p, None, 2)
        else:
            y4 = nhwc(F.conv2d(nchw(x), self.w4, None, padding=1)).contiguous()
        return K.subpixel_shortcut(y4, x, bias=self.conv.bias)

    def forward_f32(self, x32, x16):
        """On the fp32 residual stream: the phase conv reads the bf16 shadow, the interleave + bias +
        shortcut reads the fp32 stream and writes the new fp32 stream and its shadow in one pass."""
        if self.w4 is None:
            self.refresh_phase_weights()
        B, H, W, _ = x32.shape
        if self.fused_ok():
            s16 = torch.empty((B, 2 * H, 2 * W, self.w4.shape[0] // 4), dtype=torch.bfloat16, device=x32.device)
            return K.conv2x2_subpixel(x16, self.w4p, x32, bias=self.conv.bias, shadow=s16), s16
        if self.w4p is not None:
            y4 = K.conv_nhwc(x16, self.w4p, None, 2)
        else:
            y4 = nhwc(F.conv2d(nchw(x16), self.w4, None, padding=1)).contiguous()
        B, H, W, _ = x32.shape
        s16 = torch.empty((B, 2 * H, 2 * W, y4.shape[-1] // 4), dtype=torch.bfloat16, device=x32.device)
        return K.subpixel_shortcut_f32(y4, x32, bias=self.conv.bias, shadow=s16), s16

    def forward_reference(self, x):  # the literal architecture (for tests)
        up = F.interpolate(nchw(x), scale_factor=2, mode="nearest")
        y = self.conv(nhwc(up).contiguous())
        return K.upshortcut_add_(y, x.contiguous())


class DCAEDecoder(nn.Module):
    def __init__(self, latent_channels: int = 32, widths=(128, 256, 512, 512, 1024, 1024),
                 layers=(3, 3, 3, 3, 3, 3), vit_from: int = 3, scaling_factor: float = 0.41407):
        super().__init__()
        self.scaling_factor = scaling_factor
        self.latent_channels = latent_channels
        self.widths, self.layers, self.vit_from = tuple(widths), tuple(layers), vit_from
        # the fp32 residual stream in the first fp32_stages stages (lowest resolution
        # first, 32^2 .. 256^2 at 1024 px), the bf16 stream in the two high-resolution stages, which
        # carry 15/16 of the stream's bytes: pooled over 12 seeds, max |dS| 0.0164 (all bf16) -> 0.0105
        # (4 stages) vs 0.0112 (all 6), decode +3 % vs +20 % (tools/dcae_stream_probe.py,
        # profiles/r04_dcae_fp32_stages_probe.json); 0: the round-3 all-bf16 decoder (A/B)
        self.fp32_stages = min(4, len(widths))
        self.hi_res_chunk = 8     # images per call of the two high-resolution stages (see _tail)
        self.conv_in = Conv3x3(latent_channels, widths[-1])
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
        self.conv_out = Conv3x3(widths[0], 3)

    @torch.no_grad()
    def init_weights(self, seed: int = 1):
        g = torch.Generator(device=self.conv_in.weight.device).manual_seed(seed)
        for name, p in self.named_parameters():
            if p.ndim >= 2:
                if "ms_dw" in name or name.endswith("w_dw"):
                    fan_in = p.shape[0]
                elif "ms_pw" in name:
                    fan_in = p.shape[-1]
                else:
                    fan_in = p[0].numel()
                p.copy_(torch.randn(p.shape, generator=g, device=p.device) * (0.5 / math.sqrt(fan_in)))
            elif name.endswith("weight"):
                p.fill_(1.0)
            else:
                p.zero_()
        for m in self.modules():
            if isinstance(m, UpBlock):
                m.refresh_phase_weights()
            if isinstance(m, ResBlock):
                m.refresh_packed_weights()

    def _head(self, x):
        if x.shape[-1] == 128 and self.conv_out.weight.shape[0] == 3:  # norm_out + ReLU + conv_out in one pass
            no = self.norm_out
            return nchw(K.dcae_head(x, no.eps, no.weight, no.bias, self.conv_out.weight, self.conv_out.bias))
        return nchw(self.conv_out(self.norm_out(x, act="relu")))

    def _tail(self, x16, first: int):
        """Stages first.. (bf16 stream) + head; the two high-resolution stages in chunks of hi_res_chunk
        images (their kernels index one tensor with 32 bits: 8 images of 1024^2 x 128 is the largest)."""
        hi = len(self.stages) - 2
        for st in self.stages[first:hi]:
            x16 = st(x16)
        B, c = x16.shape[0], self.hi_res_chunk
        if B <= c:
            for st in self.stages[max(first, hi):]:
                x16 = st(x16)
            return self._head(x16)
        outs = []
        for s0 in range(0, B, c):
            xc = x16[s0:s0 + c]
            for st in self.stages[max(first, hi):]:
                xc = st(xc)
            outs.append(self._head(xc))
        return torch.cat(outs)

    def forward(self, z):  # z [B, 32, h, w] -> image [B, 3, 32h, 32w] (channels-last) in ~[-1, 1]
        """The low-resolution stages run on the whole batch (a call may carry more images than one chunk:
        their GEMMs / convs fill the chip better), the high-resolution stages chunk by hi_res_chunk."""
        if self.fp32_stages > 0:
            return self.forward_f32(z)
        zt = nhwc(z.to(torch.bfloat16)).contiguous()
        x = self.conv_in(zt) + zt.repeat_interleave(self.in_repeats, dim=-1)
        return self._tail(x, 0)

    def forward_f32(self, z):
        """The decoder on an fp32 residual stream: every block updates the fp32 stream x32
        in place (fused into the row norm / up-block interleave passes) and refreshes its bf16 shadow x16,
        which is what every conv / GEMM reads; the conv_in shortcut adds the fp32 latent.  The bf16
        stream rounded the decoder's residual after every block — the largest source of member-
        differential drift left after the transformer's fp32 stream.  Stages past fp32_stages run the
        bf16 stream (the high-resolution stages carry most of the stream's HBM traffic)."""
        zt = nhwc(z.to(torch.bfloat16)).contiguous()
        x32 = self.conv_in(zt).float() + nhwc(z.float()).repeat_interleave(self.in_repeats, dim=-1)
        x16 = x32.to(torch.bfloat16)
        n32 = min(self.fp32_stages, len(self.stages) - 2)
        for st in self.stages[:n32]:
            for blk in st:
                x32, x16 = blk.forward_f32(x32, x16)
        if self.fp32_stages > n32:   # fp32 stream into the high-resolution stages: unchunked (A/B only)
            for st in self.stages[n32:self.fp32_stages]:
                for blk in st:
                    x32, x16 = blk.forward_f32(x32, x16)
            n32 = self.fp32_stages
        return self._tail(x16, n32)
