"""Sana-Sprint transformer (SanaTransformer2DModel, Sana_Sprint_1.6B_1024px config) — the host
module of the perturbed LoRA linears, bf16, token-major (channels-last) throughout.

Reference: the reference loads `diffusers.SanaTransformer2DModel.from_pretrained(
"Efficient-Large-Model/Sana_Sprint_1.6B_1024px_diffusers", subfolder="transformer")` in fp32
(models/SanaSprint.py:35-39) and wraps it with PEFT.  diffusers is not installed and no weights
exist offline, so this is a from-scratch restatement of the published architecture (20 blocks,
hidden 2240 = 70 heads x 32, ReLU linear self-attention, 20 x 112 softmax cross-attention,
GLUMBConv FFN with mlp_ratio 2.5, AdaLN-single modulation with guidance embedding, RMS q/k norm
across heads).  Parity with diffusers numerics is UNPINNED (no weights / no diffusers here);
shapes, FLOPs and the LoRA target set (168 linears, D = 1,515,456 at r=2) are exact.

Non-LoRA ops run on PyTorch-ROCm (hipBLASLt GEMMs for the 1x1 convs, SDPA) or on libeggroll's
model-side fused kernels (dwconv+GLU, RMS/AdaLN row norms, gated residual); every LoRA target runs
through libeggroll's population kernel.
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field
from typing import List, Optional, Sequence, Tuple

import torch
import torch.nn.functional as F
from torch import nn

from . import kernels as K
from . import lora
from .lora import LoRALinear, bind_theta_layout


@dataclass
class SanaArch:
    in_channels: int = 32
    out_channels: int = 32
    num_attention_heads: int = 70
    attention_head_dim: int = 32
    num_layers: int = 20
    num_cross_attention_heads: int = 20
    cross_attention_head_dim: int = 112
    caption_channels: int = 2304
    mlp_ratio: float = 2.5
    norm_eps: float = 1e-6
    guidance_embeds_scale: float = 0.1
    sample_size: int = 32

    @property
    def inner_dim(self) -> int:
        return self.num_attention_heads * self.attention_head_dim


SANA_SPRINT_1_6B = SanaArch()
SANA_LORA_TARGETS = ["to_q", "to_k", "to_v", "to_out.0", "linear_1", "linear_2", "proj_out", "linear"]  # unifed_es.py:391


class RMSNorm(nn.Module):
    def __init__(self, dim: int, eps: float = 1e-5, bias: bool = False):
        super().__init__()
        self.eps = eps
        self.weight = nn.Parameter(torch.ones(dim, dtype=torch.bfloat16), requires_grad=False)
        self.bias = nn.Parameter(torch.zeros(dim, dtype=torch.bfloat16), requires_grad=False) if bias else None

    def forward(self, x, act=None):
        return K.rownorm(x.contiguous(), self.eps, layer=False, w=self.weight, b=self.bias, act=act)


def timestep_embedding(t: torch.Tensor, dim: int = 256, max_period: float = 10000.0) -> torch.Tensor:
    """diffusers get_timestep_embedding(flip_sin_to_cos=True, downscale_freq_shift=0)."""
    half = dim // 2
    exponent = -math.log(max_period) * torch.arange(half, dtype=torch.float32, device=t.device) / half
    emb = t.float()[:, None] * torch.exp(exponent)[None, :]
    return torch.cat([torch.cos(emb), torch.sin(emb)], dim=-1)


class TimestepEmbedding(nn.Module):
    def __init__(self, in_dim: int, dim: int):
        super().__init__()
        self.linear_1 = LoRALinear(in_dim, dim, lora=False)
        self.linear_2 = LoRALinear(dim, dim, lora=False)

    def forward(self, x):
        return self.linear_2(F.silu(self.linear_1(x)))


class CombinedTimestepGuidanceEmbeddings(nn.Module):
    """SanaCombinedTimestepGuidanceEmbeddings: returns (6*D modulation, D embedded timestep)."""

    def __init__(self, dim: int):
        super().__init__()
        self.timestep_embedder = TimestepEmbedding(256, dim)
        self.guidance_embedder = TimestepEmbedding(256, dim)
        self.linear = LoRALinear(dim, 6 * dim, lora=False)

    def forward(self, timestep, guidance, fp32: bool = False):
        """fp32: the whole chain in fp32 (LoRALinear.forward_fp32; B rows, negligible cost) — it sets every
        token's AdaLN modulation, and its bf16 rounding was member-differential error."""
        if fp32:
            lf = lambda m, v: m.forward_fp32(v)  # noqa: E731
            t = lf(self.timestep_embedder.linear_2, F.silu(lf(self.timestep_embedder.linear_1, timestep_embedding(timestep))))
            g = lf(self.guidance_embedder.linear_2, F.silu(lf(self.guidance_embedder.linear_1, timestep_embedding(guidance))))
            cond = t + g
            return lf(self.linear, F.silu(cond)), cond
        t = self.timestep_embedder(timestep_embedding(timestep).to(torch.bfloat16))
        g = self.guidance_embedder(timestep_embedding(guidance).to(torch.bfloat16))
        cond = t + g
        return self.linear(F.silu(cond)), cond


class TextProjection(nn.Module):
    """PixArtAlphaTextProjection: linear_1 -> GELU(tanh) -> linear_2."""

    def __init__(self, in_features: int, hidden: int):
        super().__init__()
        self.linear_1 = LoRALinear(in_features, hidden, lora=False)
        self.linear_2 = LoRALinear(hidden, hidden, lora=False)

    def forward(self, x):
        return self.linear_2(F.gelu(self.linear_1(x), approximate="tanh"))


class LinearSelfAttention(nn.Module):
    """attn1 with SanaLinearAttnProcessor2_0 (ReLU kernel, fp32 accumulation)."""

    def __init__(self, dim: int, heads: int, head_dim: int, eps: float = 1e-5):
        super().__init__()
        if head_dim != 32:
            raise ValueError("LinearSelfAttention: eggroll_linear_attention is specialised for head_dim 32")
        self.heads, self.head_dim = heads, head_dim
        inner = heads * head_dim
        self.norm_q = RMSNorm(inner, eps)
        self.norm_k = RMSNorm(inner, eps)
        self.to_q = LoRALinear(dim, inner, bias=False, lora=False)
        self.to_k = LoRALinear(dim, inner, bias=False, lora=False)
        self.to_v = LoRALinear(dim, inner, bias=False, lora=False)
        self.to_out = nn.ModuleList([LoRALinear(inner, dim, bias=True, lora=False)])

    def forward(self, x, res=None, gate=None, shadow=None):  # x [B, N, D]
        """With res / gate: returns res += gate[image] * attn1(x), the gated residual fused into
        to_out's GEMM epilogue (the block's `x + gate_msa * attn_output`); an fp32 res is the fp32
        residual stream (gate fp32, shadow = its bf16 copy written in the same epilogue)."""
        B, N, D = x.shape
        Tq, Tk, Tv = lora.shared_projection([self.to_q, self.to_k, self.to_v], x)   # X read once for 3 LoRAs
        q = self.norm_q(self.to_q(x, T=Tq), act="relu").view(B * N, -1)   # RMS norm + ReLU fused
        k = self.norm_k(self.to_k(x, T=Tk), act="relu").view(B * N, -1)
        v = self.to_v(x, T=Tv).view(B * N, -1)
        o = K.linear_attention(q, k, v, B, N, self.heads, self.head_dim, relu_qk=False)
        if res is not None:
            epi = "gated32" if res.dtype == torch.float32 else "gated"
            return self.to_out[0](o.view(B, N, -1), epi=epi, res=res, gate=gate, rows_per_group=N, shadow=shadow)
        return self.to_out[0](o.view(B, N, -1))


class CrossAttention(nn.Module):
    """attn2: softmax cross-attention over the 300 caption tokens (SanaAttnProcessor2_0)."""

    def __init__(self, dim: int, heads: int, head_dim: int, eps: float = 1e-5):
        super().__init__()
        self.heads, self.head_dim = heads, head_dim
        inner = heads * head_dim
        self.norm_q = RMSNorm(inner, eps)
        self.norm_k = RMSNorm(inner, eps)
        self.to_q = LoRALinear(dim, inner, bias=True, lora=False)
        self.to_k = LoRALinear(dim, inner, bias=True, lora=False)
        self.to_v = LoRALinear(dim, inner, bias=True, lora=False)
        self.to_out = nn.ModuleList([LoRALinear(inner, dim, bias=True, lora=False)])
        self.pad_head_dim = True   # pad the SDPA head dim to a multiple of 64 (exact, see forward)
        self.use_kernel = True     # eggroll_cross_attention where it applies (head dim 112, L <= 320)

    def forward(self, x, enc, mask_bias, enc_index=None, res=None):
        """x [B,N,D]; enc [U,L,D] caption rows; mask_bias [U, L] additive caption mask per caption row;
        enc_index [B] (image -> caption row, None: U == B).  Images that share a caption share its k / v
        rows, so to_k / to_v (and the caption projection before them) run once per distinct caption.
        Head dim 112 with L <= 320 runs libeggroll's MFMA cross-attention (k / v read through
        enc_index, q / o in the projection layout); otherwise SDPA on gathered k / v."""
        B, N, _ = x.shape
        U, L = enc.shape[0], enc.shape[1]
        hd = self.head_dim
        if self.use_kernel and hd == 112 and L <= 320:
            q = self.norm_q(self.to_q(x)).view(B * N, -1)
            Tk, Tv = lora.shared_projection([self.to_k, self.to_v], enc)
            k = self.norm_k(self.to_k(enc, T=Tk)).view(U * L, -1)
            v = self.to_v(enc, T=Tv).view(U * L, -1)
            o = K.cross_attention(q, k, v, B, N, self.heads, hd, L, hd ** -0.5, bias=mask_bias.contiguous(),
                                  enc_index=enc_index).view(B, N, -1)
            if res is not None:   # res += to_out(o): the block's residual add fused into the GEMM epilogue
                return self.to_out[0](o, epi="res32" if res.dtype == torch.float32 else "res", res=res)
            return self.to_out[0](o)
        q = self.norm_q(self.to_q(x)).view(B, N, self.heads, hd)
        k = self.norm_k(self.to_k(enc)).view(U, L, self.heads, hd)
        v = self.to_v(enc).view(U, L, self.heads, hd)
        mask_bias = (mask_bias if enc_index is None else mask_bias.index_select(0, enc_index)).view(B, 1, 1, L)
        pad = (-hd) % 64 if self.pad_head_dim else 0
        if pad:
            # SDPA at head dim 112 runs ~2.7x slower than at 128 on gfx950; zero-padded dims add exact
            # zeros to q.k and give zero output columns, so with the 1/sqrt(112) scale passed explicitly
            # the result is bit-identical (tools/xattn_pad_probe.py, tests/test_gpu_engine.py)
            q, k, v = (F.pad(t, (0, pad)) for t in (q, k, v))
        if enc_index is not None:
            k, v = k.index_select(0, enc_index), v.index_select(0, enc_index)
        o = F.scaled_dot_product_attention(q.transpose(1, 2), k.transpose(1, 2), v.transpose(1, 2),
                                           attn_mask=mask_bias, scale=hd ** -0.5)
        if pad:
            o = o[..., :hd]
        o = o.transpose(1, 2).reshape(B, N, -1)
        if res is not None:   # res += to_out(o): the block's residual add fused into the GEMM epilogue
            return self.to_out[0](o, epi="res32" if res.dtype == torch.float32 else "res", res=res)
        return self.to_out[0](o)


class GLUMBConv(nn.Module):
    """1x1 conv -> SiLU -> 3x3 depthwise -> GLU(SiLU gate) -> 1x1 conv (token-major layout)."""

    def __init__(self, dim: int, hidden: int):
        super().__init__()
        self.hidden = hidden
        self.w_inv = nn.Parameter(torch.empty(2 * hidden, dim, dtype=torch.bfloat16), requires_grad=False)
        self.b_inv = nn.Parameter(torch.zeros(2 * hidden, dtype=torch.bfloat16), requires_grad=False)
        self.w_dw = nn.Parameter(torch.empty(9, 2 * hidden, dtype=torch.bfloat16), requires_grad=False)  # [tap][C]
        self.b_dw = nn.Parameter(torch.zeros(2 * hidden, dtype=torch.bfloat16), requires_grad=False)
        self.w_point = nn.Parameter(torch.empty(dim, hidden, dtype=torch.bfloat16), requires_grad=False)

    def _point_weight(self, kp: int) -> torch.Tensor:
        """w_point zero-padded to kp input channels (cached; rebuilt when w_point changes)."""
        key = (self.w_point._version, self.w_point.data_ptr(), kp)
        if getattr(self, "_wp_key", None) != key:
            self._wp = F.pad(self.w_point.detach(), (0, kp - self.hidden)).contiguous()
            self._wp_key = key
        return self._wp

    def forward(self, x, H: int, W: int, res=None, gate=None):  # x [B, N, D]
        """res / gate (optional): the block's gated residual x += gate_mlp * ff(x) fused into the
        point conv's GEMM epilogue ("gated32" on the fp32 stream, "gated" on bf16); returns res."""
        B, N, D = x.shape
        # 1x1 conv on the 8-phase GEMM, then SiLU -> dw3x3 -> GLU in the depthwise conv (SiLU applied once
        # per staged element); lora.SILU_IN_GEMM moves the SiLU into the GEMM epilogue instead — the same
        # bits (silu of the bf16-rounded output), measured 1.2 % slower per FFN since round 5's cheaper
        # depthwise staging (tools/silu_split_probe.py, profiles/r09q_silu_placement.log)
        kp = -(-self.hidden // 64) * 64     # 5600 -> 5632: the GEMM's k-step is 64
        if lora.FUSE_EPILOGUES and lora.SILU_IN_GEMM:
            h = K.lora_linear_pop_epi(x.reshape(B * N, D), self.w_inv, self.b_inv, None, 0, 0, 0, 0.0, B * N, "silu")
            g = K.dwconv_nhwc(h.view(B, H, W, -1), self.w_dw, self.b_dw, 3, pre_silu=False, glu=True, ldo=kp)
        else:
            h = K.lora_linear_pop(x.reshape(B * N, D), self.w_inv, self.b_inv, None, 0, 0, 0, 0.0, B * N)
            g = K.dwconv_nhwc(h.view(B, H, W, -1), self.w_dw, self.b_dw, 3, pre_silu=True, glu=True, ldo=kp)
        # 1x1 point conv on the 8-phase GEMM: the GLU output's zero pad channels meet the weight's zero
        # pad columns (exact), so hipBLASLt's K = 5600 GEMM and its separate residual pass are gone
        g, wp = g.view(B * N, kp), self._point_weight(kp)
        if res is None:
            return K.lora_linear_pop(g, wp, None, None, 0, 0, 0, 0.0, B * N).view(B, N, D)
        epi = "gated32" if res.dtype == torch.float32 else "gated"
        K.lora_linear_pop_epi(g, wp, None, None, 0, 0, 0, 0.0, B * N, epi, res=res.view(B * N, D), gate=gate,
                              rows_per_group=N)
        return res


class SanaBlock(nn.Module):
    def __init__(self, a: SanaArch):
        super().__init__()
        D = a.inner_dim
        self.eps = a.norm_eps
        self.attn1 = LinearSelfAttention(D, a.num_attention_heads, a.attention_head_dim)
        self.attn2 = CrossAttention(D, a.num_cross_attention_heads, a.cross_attention_head_dim)
        self.ff = GLUMBConv(D, int(a.mlp_ratio * D))
        self.scale_shift_table = nn.Parameter(torch.randn(6, D).div(D ** 0.5).to(torch.bfloat16), requires_grad=False)

    def forward_fp32(self, x32, x16, enc, mask_bias, timestep, H, W, enc_index=None):
        """The block on the fp32 residual stream x32 (updated in place; x16 = its bf16 shadow, the
        GEMM operand of attn2's to_q) with the fp32 AdaLN modulation: every update of x is an fp32
        add (fused into the GEMM epilogues / eggroll_gated_residual_f32) instead of a bf16 rounding,
        the norms read x32 directly.  DESIGN §3.2: the bf16 residual stream was the largest single
        source of member-differential drift in the transformer at sigma = 1e-2."""
        B, N, D = x32.shape
        mods = self.scale_shift_table.float()[None] + timestep.view(B, 6, -1)
        n = K.rownorm(x32, self.eps, layer=True, mscale=mods[:, 1], mshift=mods[:, 0], rows_per_group=N)
        if lora.FUSE_EPILOGUES:
            self.attn1(n, res=x32, gate=mods[:, 2], shadow=x16)    # x32 += gate_msa * attn1(n); x16 = bf16(x32)
            self.attn2(x16, enc, mask_bias, enc_index, res=x32)    # x32 += attn2(x16)
        else:                                                      # the same ops unfused (bit-identical)
            K.gated_residual_f32_(x32, self.attn1(n), mods[:, 2], rows_per_group=N, shadow=x16)
            K.gated_residual_f32_(x32, self.attn2(x16, enc, mask_bias, enc_index), None, rows_per_group=N)
        n = K.rownorm(x32, self.eps, layer=True, mscale=mods[:, 4], mshift=mods[:, 3], rows_per_group=N)
        if lora.FUSE_EPILOGUES:
            self.ff(n, H, W, res=x32, gate=mods[:, 5])             # x32 += gate_mlp * ff(n)
        else:
            K.gated_residual_f32_(x32, self.ff(n, H, W), mods[:, 5], rows_per_group=N)
        return x32

    def forward(self, x, enc, mask_bias, timestep, H, W, enc_index=None):
        B, N, D = x.shape
        # [B, 6, D]: shift_msa, scale_msa, gate_msa, shift_mlp, scale_mlp, gate_mlp
        mods = (self.scale_shift_table[None] + timestep.view(B, 6, -1)).contiguous()
        n = K.rownorm(x, self.eps, layer=True, mscale=mods[:, 1], mshift=mods[:, 0], rows_per_group=N)
        if lora.FUSE_EPILOGUES:
            self.attn1(n, res=x, gate=mods[:, 2])             # x += gate_msa * attn1(n), in to_out's epilogue
            self.attn2(x, enc, mask_bias, enc_index, res=x)   # x = x + attn2(x): in to_out's epilogue
        else:                                                 # the same ops unfused (bit-identical)
            K.gated_residual_(x, self.attn1(n), mods[:, 2], rows_per_group=N)
            x = x + self.attn2(x, enc, mask_bias, enc_index)
        n = K.rownorm(x, self.eps, layer=True, mscale=mods[:, 4], mshift=mods[:, 3], rows_per_group=N)
        if lora.FUSE_EPILOGUES:
            self.ff(n, H, W, res=x, gate=mods[:, 5])               # x += gate_mlp * ff(n)
        else:
            K.gated_residual_(x, self.ff(n, H, W), mods[:, 5], rows_per_group=N)
        return x


class SanaTransformer2DModel(nn.Module):
    def __init__(self, a: SanaArch = SANA_SPRINT_1_6B):
        super().__init__()
        self.config = a
        D = a.inner_dim
        # module registration order follows diffusers (theta layout = parameter order)
        self.patch_w = nn.Parameter(torch.empty(D, a.in_channels, dtype=torch.bfloat16), requires_grad=False)
        self.patch_b = nn.Parameter(torch.zeros(D, dtype=torch.bfloat16), requires_grad=False)
        self.time_embed = CombinedTimestepGuidanceEmbeddings(D)
        self.caption_projection = TextProjection(a.caption_channels, D)
        self.caption_norm = RMSNorm(D, 1e-5)
        self.transformer_blocks = nn.ModuleList([SanaBlock(a) for _ in range(a.num_layers)])
        self.scale_shift_table = nn.Parameter(torch.randn(2, D).div(D ** 0.5).to(torch.bfloat16), requires_grad=False)
        self.proj_out = LoRALinear(D, a.out_channels, lora=False)
        # opt-in (exact, see forward): off by default so the bench runs the reference's full 300-token
        # cross-attention and caption projection (measured +0.8 % epoch throughput on the synthetic prompts)
        self.trim_caption_padding = False
        # fp32 residual stream + fp32 time embedding / modulation / output projection;
        # False: the round-3 all-bf16 path (kept for A/B)
        self.fp32_stream = True

    @torch.no_grad()
    def init_weights(self, seed: int = 0):
        """Synthetic frozen weights (no checkpoints offline): N(0, 1/fan_in) so activations stay O(1)."""
        g = torch.Generator(device=self.patch_w.device).manual_seed(seed)
        for name, p in self.named_parameters():
            if p.requires_grad:
                continue
            if name.endswith("scale_shift_table"):
                p.copy_(torch.randn(p.shape, generator=g, device=p.device).div(p.shape[-1] ** 0.5))
            elif name.endswith("w_dw"):
                p.copy_(torch.randn(p.shape, generator=g, device=p.device) / 3.0)   # fan_in 9
            elif p.ndim >= 2:
                fan_in = p[0].numel()
                std = 1.0 / math.sqrt(fan_in)
                if name.endswith("to_out.0.weight") or name.endswith("w_point") or "proj_out" in name:
                    std *= 0.5
                p.copy_(torch.randn(p.shape, generator=g, device=p.device) * std)
            elif name.endswith("weight"):
                p.fill_(1.0)
            else:
                p.zero_()

    def forward(self, hidden_states, timestep, encoder_hidden_states, encoder_attention_mask, guidance,
                enc_index=None):
        """enc_index (optional, build-specific): [B] image -> row of encoder_hidden_states /
        encoder_attention_mask, which then hold only the DISTINCT captions (the caption projection,
        caption norm and every block's to_k / to_v run once per distinct caption).  None: one caption
        row per image, as diffusers' SanaTransformer2DModel."""
        B, C, H, W = hidden_states.shape
        a = self.config
        f32 = self.fp32_stream
        if f32:   # PatchEmbed (p = 1) in fp32 (K = 32): the fp32 residual stream starts here
            x = F.linear(hidden_states.float().permute(0, 2, 3, 1).reshape(B, H * W, C), self.patch_w.float(),
                         self.patch_b.float()).contiguous()
            x16 = torch.empty(x.shape, dtype=torch.bfloat16, device=x.device)
        else:
            x = hidden_states.to(torch.bfloat16).permute(0, 2, 3, 1).reshape(B, H * W, C)
            x = F.linear(x, self.patch_w, self.patch_b).contiguous()                      # PatchEmbed (p = 1)
        timestep6, emb_t = self.time_embed(timestep, guidance, fp32=f32)
        if self.trim_caption_padding and encoder_attention_mask is not None:
            # Caption columns that are padding for EVERY image carry a -10000 bias: their softmax weight
            # underflows to exactly 0, so dropping them (and their caption-projection / k / v rows) is
            # exact.  Only applied when every image keeps at least one valid token (an all-masked row
            # would otherwise softmax uniformly over the padding).  One host read per forward.
            valid = encoder_attention_mask != 0
            cols = valid.any(0).nonzero()
            if cols.numel() and bool(valid.any(1).all()):
                L_eff = int(cols.max()) + 1
                encoder_hidden_states = encoder_hidden_states[:, :L_eff]
                encoder_attention_mask = encoder_attention_mask[:, :L_eff]
        enc = self.caption_projection(encoder_hidden_states.to(torch.bfloat16))
        enc = self.caption_norm(enc)
        mask_bias = (1.0 - encoder_attention_mask.to(torch.bfloat16)) * -10000.0   # [U, L], per caption row
        if f32:
            for blk in self.transformer_blocks:
                blk.forward_fp32(x, x16, enc, mask_bias, timestep6, H, W, enc_index)
            mods = self.scale_shift_table.float()[None] + emb_t[:, None]          # [B, 2, D]: shift, scale
            n = K.rownorm(x, a.norm_eps, layer=True, mscale=mods[:, 1], mshift=mods[:, 0], rows_per_group=H * W)
            x = self.proj_out.forward_fp32(n)                                      # fp32 output (the SCM math)
            return x.view(B, H, W, a.out_channels).permute(0, 3, 1, 2)
        for blk in self.transformer_blocks:
            x = blk(x, enc, mask_bias, timestep6, H, W, enc_index)
        mods = (self.scale_shift_table[None] + emb_t[:, None]).contiguous()     # [B, 2, D]: shift, scale
        x = K.rownorm(x, a.norm_eps, layer=True, mscale=mods[:, 1], mshift=mods[:, 0], rows_per_group=H * W)
        x = self.proj_out(x)
        return x.view(B, H, W, a.out_channels).permute(0, 3, 1, 2)


def attach_lora(model: nn.Module, r: int, alpha: float, targets: Sequence[str]) -> int:
    """get_peft_model equivalent (es_backend.py:193-200): enable LoRA on every LoRALinear whose
    qualified name equals or ends with '.<target>' (PEFT suffix matching)."""
    n = 0
    for name, m in model.named_modules():
        if isinstance(m, LoRALinear) and any(name == t or name.endswith("." + t) for t in targets):
            dev = m.weight.device
            m.r, m.scale = r, float(alpha) / r
            m.lora_A = nn.Module()
            m.lora_A.weight = nn.Parameter(torch.zeros(r, m.in_features, device=dev))
            m.lora_B = nn.Module()
            m.lora_B.weight = nn.Parameter(torch.zeros(m.out_features, r, device=dev))
            n += 1
    bind_theta_layout(model)
    return n


def sana_lora_shapes(a: SanaArch = SANA_SPRINT_1_6B, r: int = 2, alpha: float = 8.0,
                     targets: Sequence[str] = tuple(SANA_LORA_TARGETS)) -> List[Tuple[int, ...]]:
    """theta layout (trainable shapes in module.parameters() order, utills.py:141-152) of the
    LoRA'd transformer, built on the meta device: no weights are allocated."""
    with torch.device("meta"):
        model = SanaTransformer2DModel(a)
        attach_lora(model, r, alpha, targets)
    return [tuple(p.shape) for p in model.parameters() if p.requires_grad]
