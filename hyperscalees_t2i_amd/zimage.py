"""Z-Image-Turbo transformer (diffusers ZImageTransformer2DModel, Tongyi-MAI/Z-Image-Turbo config) — the
host module of BASELINE configs[3]'s perturbed LoRA linears, bf16, token-major throughout.

Reference: `ZImagePipeline.from_pretrained("Tongyi-MAI/Z-Image-Turbo")` wrapped with PEFT on the targets
to_q, to_k, to_v, linear, w1, w2, w3 (models/zImageTurbo.py:96-101, es_backend.py:566-584,
unifed_es.py:482-485), generated in bf16 at 384 px with 7 flow-matching steps and no guidance
(unifed_es.py:413-417).  diffusers is not installed and no weights exist offline, so this is a
from-scratch restatement of the published single-stream DiT ("S3-DiT"): 3840 wide, 30 heads x 128,
2 noise-refiner blocks (image tokens, AdaLN-modulated), 2 context-refiner blocks (caption tokens,
unmodulated), 30 main blocks over the concatenated [image | caption] sequence, SwiGLU FFN 10240,
RMSNorm everywhere with tanh-gated sandwich norms, RMS q/k norm per head, 3-axis RoPE (32/48/48,
theta 256), a 256-wide timestep embedding feeding every block's 4-way modulation.  Parity with
diffusers numerics and the exact module tree are UNPINNED (no diffusers, no checkpoint here): the
shapes, FLOPs, token counts and the LoRA target set follow the published config, which is what the
throughput of configs[3] depends on.

Every linear runs on libeggroll's population GEMM (LoRA'd or plain); the q/k norm + RoPE on
`eggroll_qk_norm_rope` (one in-place pass per tensor); every RMSNorm / modulation / gated residual on
`eggroll_rownorm`; attention on `eggroll_flash_attention` (head dim 128, no mask); the FFN's
silu(w1 x) on the GEMM's SiLU epilogue.
"""
from __future__ import annotations

import math
from dataclasses import dataclass
from typing import List, Optional, Sequence, Tuple

import torch
import torch.nn.functional as F
from torch import nn

from . import kernels as K
from . import lora
from .lora import LoRALinear
from .sana import attach_lora, timestep_embedding


@dataclass
class ZImageArch:
    in_channels: int = 16
    patch: int = 2
    dim: int = 3840
    n_layers: int = 30
    n_refiner_layers: int = 2
    n_heads: int = 30
    ffn: int = 10240             # int(dim / 3 * 8)
    norm_eps: float = 1e-5
    cap_feat_dim: int = 2560     # Qwen3-4B hidden size
    adaln_dim: int = 256         # min(dim, ADALN_EMBED_DIM)
    t_mid: int = 1024
    t_scale: float = 1000.0
    rope_theta: float = 256.0
    axes_dims: Tuple[int, int, int] = (32, 48, 48)
    seq_multiple: int = 32       # caption / image token counts are padded to a multiple of this

    @property
    def head_dim(self) -> int:
        return self.dim // self.n_heads

    @property
    def patch_dim(self) -> int:
        return self.patch * self.patch * self.in_channels


ZIMAGE_TURBO = ZImageArch()
ZIMAGE_LORA_TARGETS = ["to_q", "to_k", "to_v", "linear", "w1", "w2", "w3"]   # unifed_es.py:485


class RMSNorm(nn.Module):
    def __init__(self, dim: int, eps: float):
        super().__init__()
        self.eps = eps
        self.weight = nn.Parameter(torch.ones(dim, dtype=torch.bfloat16), requires_grad=False)


def rope_tables(arch: ZImageArch, pos: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor]:
    """pos [..., 3] integer positions (caption index / row / column axes) -> cos, sin [..., head_dim / 2]
    fp32: axis a covers axes_dims[a] / 2 rotation pairs with frequencies theta^(-2i / axes_dims[a])."""
    cs, ss = [], []
    for a, d in enumerate(arch.axes_dims):
        inv = 1.0 / (arch.rope_theta ** (torch.arange(0, d, 2, dtype=torch.float64, device=pos.device) / d))
        ang = pos[..., a].double()[..., None] * inv
        cs.append(torch.cos(ang))
        ss.append(torch.sin(ang))
    return torch.cat(cs, -1).float(), torch.cat(ss, -1).float()


def apply_rope(x: torch.Tensor, cos: torch.Tensor, sin: torch.Tensor, n_rep: int) -> torch.Tensor:
    """x [n_rep * b, S, H, D] bf16; cos / sin [b, S, D/2] (shared by the n_rep member copies): adjacent
    element pairs rotate as complex numbers (x0 + i x1) * (cos + i sin), in fp32, rounded once."""
    B, S, H, D = x.shape
    xf = x.view(n_rep, B // n_rep, S, H, D // 2, 2).float()
    c, s = cos[None, :, :, None, :], sin[None, :, :, None, :]
    x0, x1 = xf[..., 0], xf[..., 1]
    return torch.stack((x0 * c - x1 * s, x0 * s + x1 * c), -1).to(torch.bfloat16).view(B, S, H, D)


class ZAttention(nn.Module):
    def __init__(self, a: ZImageArch):
        super().__init__()
        self.heads, self.hd = a.n_heads, a.head_dim
        self.to_q = LoRALinear(a.dim, a.dim, bias=False, lora=False)
        self.to_k = LoRALinear(a.dim, a.dim, bias=False, lora=False)
        self.to_v = LoRALinear(a.dim, a.dim, bias=False, lora=False)
        self.norm_q = RMSNorm(a.head_dim, a.norm_eps)
        self.norm_k = RMSNorm(a.head_dim, a.norm_eps)
        self.to_out = nn.ModuleList([LoRALinear(a.dim, a.dim, bias=False, lora=False)])
        self.use_kernel = True   # eggroll_qk_norm_rope + eggroll_flash_attention; False: torch forms (A/B, tests)

    def forward(self, x, cos, sin, n_rep: int, key_bias: Optional[torch.Tensor]):
        """x [B, S, dim]; key_bias [B, 1, 1, S] additive (batch padding) or None."""
        B, S, D = x.shape
        Tq, Tk, Tv = lora.shared_projection([self.to_q, self.to_k, self.to_v], x)   # X read once for 3 LoRAs
        q, k = self.to_q(x, T=Tq), self.to_k(x, T=Tk)
        if self.use_kernel and self.hd == 128:   # norm + RoPE in one in-place pass per tensor
            c2, s2 = cos.reshape(-1, cos.shape[-1]), sin.reshape(-1, sin.shape[-1])
            K.qk_norm_rope_(q.view(-1, D), self.norm_q.weight, self.norm_q.eps, c2, s2, self.heads)
            K.qk_norm_rope_(k.view(-1, D), self.norm_k.weight, self.norm_k.eps, c2, s2, self.heads)
            q, k = q.view(B, S, self.heads, self.hd), k.view(B, S, self.heads, self.hd)
        else:
            q = K.rownorm(q.view(-1, self.hd), self.norm_q.eps, w=self.norm_q.weight)
            k = K.rownorm(k.view(-1, self.hd), self.norm_k.eps, w=self.norm_k.weight)
            q = apply_rope(q.view(B, S, self.heads, self.hd), cos, sin, n_rep)
            k = apply_rope(k.view(B, S, self.heads, self.hd), cos, sin, n_rep)
        v = self.to_v(x, T=Tv).view(B, S, self.heads, self.hd)
        if self.use_kernel and self.hd == 128 and key_bias is None:   # eggroll_flash_attention
            o = K.flash_attention(q, k, v, self.hd ** -0.5)
            return self.to_out[0](o.view(B, S, D))
        o = F.scaled_dot_product_attention(q.transpose(1, 2), k.transpose(1, 2), v.transpose(1, 2),
                                           attn_mask=key_bias, scale=self.hd ** -0.5)
        return self.to_out[0](o.transpose(1, 2).reshape(B, S, D))


class ZFeedForward(nn.Module):
    """w2(silu(w1 x) * w3 x); silu(w1 x) comes out of w1's SiLU epilogue (the same bf16 values as torch's
    silu of the rounded output) and the product out of w3's multiply epilogue (bf16(h * y), torch's mul)."""

    def __init__(self, a: ZImageArch):
        super().__init__()
        self.w1 = LoRALinear(a.dim, a.ffn, bias=False, lora=False)
        self.w2 = LoRALinear(a.ffn, a.dim, bias=False, lora=False)
        self.w3 = LoRALinear(a.dim, a.ffn, bias=False, lora=False)

    def forward(self, x):
        h = self.w1(x, epi="silu")
        self.w3(x, epi="mul", res=h)          # h *= w3 x in the w3 GEMM's epilogue
        return self.w2(h)


class ZBlock(nn.Module):
    """ZImageTransformerBlock: sandwich RMSNorms around attention and FFN; with modulation the
    pre-norms are scaled by (1 + scale) and the post-norm branches gated by tanh(gate) from
    adaLN_modulation(t_emb) = [scale_msa | gate_msa | scale_mlp | gate_mlp]."""

    def __init__(self, a: ZImageArch, modulation: bool):
        super().__init__()
        self.dim = a.dim
        self.attention = ZAttention(a)
        self.feed_forward = ZFeedForward(a)
        self.attention_norm1 = RMSNorm(a.dim, a.norm_eps)
        self.ffn_norm1 = RMSNorm(a.dim, a.norm_eps)
        self.attention_norm2 = RMSNorm(a.dim, a.norm_eps)
        self.ffn_norm2 = RMSNorm(a.dim, a.norm_eps)
        self.modulation = modulation
        if modulation:
            self.adaLN_modulation = nn.ModuleList([LoRALinear(a.adaln_dim, 4 * a.dim, bias=True, lora=False)])

    def forward(self, x, cos, sin, n_rep: int, key_bias=None, t_emb=None):
        """x [B, S, dim] bf16, updated in place (the residual adds are fused into the post-norm passes)."""
        B, S, D = x.shape
        rows = B * S
        n1, n2, f1, f2 = self.attention_norm1, self.attention_norm2, self.ffn_norm1, self.ffn_norm2
        if self.modulation:
            # one modulation row for every token (all images share the step's timestep); fp32, so the gate
            # enters the fused pass as mscale = tanh(gate) - 1: norm * w * (1 + mscale) = gate * norm * w
            m = self.adaLN_modulation[0].forward_fp32(t_emb).view(4, D)
            s_msa, g_msa, s_mlp, g_mlp = m[0:1], torch.tanh(m[1:2]) - 1.0, m[2:3], torch.tanh(m[3:4]) - 1.0
        else:
            s_msa = g_msa = s_mlp = g_mlp = None
        a = self.attention(K.rownorm(x, n1.eps, w=n1.weight, mscale=s_msa, rows_per_group=rows), cos, sin, n_rep,
                           key_bias)
        K.rownorm(a, n2.eps, w=n2.weight, mscale=g_msa, rows_per_group=rows, res=x, out=x)
        f = self.feed_forward(K.rownorm(x, f1.eps, w=f1.weight, mscale=s_mlp, rows_per_group=rows))
        K.rownorm(f, f2.eps, w=f2.weight, mscale=g_mlp, rows_per_group=rows, res=x, out=x)
        return x


class TimestepEmbedder(nn.Module):
    def __init__(self, a: ZImageArch):
        super().__init__()
        self.mlp = nn.ModuleList([LoRALinear(256, a.t_mid, bias=True, lora=False), nn.SiLU(),
                                  LoRALinear(a.t_mid, a.adaln_dim, bias=True, lora=False)])

    def forward(self, t):  # [n] model time in [0, 1] (pre-scaled by t_scale) -> [n, adaln_dim] fp32
        h = self.mlp[0].forward_fp32(timestep_embedding(t))
        return self.mlp[2].forward_fp32(F.silu(h))


class FinalLayer(nn.Module):
    def __init__(self, a: ZImageArch):
        super().__init__()
        self.linear = LoRALinear(a.dim, a.patch_dim, bias=True, lora=False)
        self.adaLN_modulation = nn.ModuleList([nn.SiLU(), LoRALinear(a.adaln_dim, a.dim, bias=True, lora=False)])

    def forward(self, x, t_emb):  # x [B, N, dim] (a strided view is fine) -> [B, N, patch_dim]
        B, N, D = x.shape
        scale = self.adaLN_modulation[1].forward_fp32(F.silu(t_emb)).view(1, D)
        n = K.rownorm(x.reshape(B * N, D), 1e-6, layer=True, mscale=scale, rows_per_group=B * N)
        return self.linear(n.view(B, N, D))


class ZImageTransformer2DModel(nn.Module):
    def __init__(self, a: ZImageArch = ZIMAGE_TURBO):
        super().__init__()
        self.config = a
        # registration order follows diffusers' __init__ (the theta layout is parameter order)
        self.all_x_embedder = nn.ModuleDict({f"{a.patch}-1": LoRALinear(a.patch_dim, a.dim, bias=True, lora=False)})
        self.all_final_layer = nn.ModuleDict({f"{a.patch}-1": FinalLayer(a)})
        self.noise_refiner = nn.ModuleList([ZBlock(a, True) for _ in range(a.n_refiner_layers)])
        self.context_refiner = nn.ModuleList([ZBlock(a, False) for _ in range(a.n_refiner_layers)])
        self.t_embedder = TimestepEmbedder(a)
        self.cap_embedder = nn.ModuleList([RMSNorm(a.cap_feat_dim, a.norm_eps),
                                           LoRALinear(a.cap_feat_dim, a.dim, bias=True, lora=False)])
        self.x_pad_token = nn.Parameter(torch.zeros(1, a.dim, dtype=torch.bfloat16), requires_grad=False)
        self.cap_pad_token = nn.Parameter(torch.zeros(1, a.dim, dtype=torch.bfloat16), requires_grad=False)
        self.layers = nn.ModuleList([ZBlock(a, True) for _ in range(a.n_layers)])

    @torch.no_grad()
    def init_weights(self, seed: int = 0):
        """Synthetic frozen weights: N(0, 1/fan_in), the residual-branch outputs (to_out, w2) and the
        modulation tables at half that, norms at 1."""
        g = torch.Generator(device=self.x_pad_token.device).manual_seed(seed)
        for name, p in self.named_parameters():
            if p.requires_grad:
                continue
            if name.endswith("pad_token"):
                p.copy_(torch.randn(p.shape, generator=g, device=p.device) * 0.02)
            elif p.ndim >= 2:
                std = 1.0 / math.sqrt(p.shape[1])
                if name.endswith("to_out.0.weight") or name.endswith("w2.weight") or "adaLN" in name:
                    std *= 0.5
                p.copy_(torch.randn(p.shape, generator=g, device=p.device) * std)
            elif name.endswith("norm1.weight") or name.endswith("norm2.weight") or "norm_" in name or \
                    name.startswith("cap_embedder.0"):
                p.fill_(1.0)
            else:
                p.zero_()

    # ---- geometry ------------------------------------------------------------------
    def patchify(self, lat: torch.Tensor) -> torch.Tensor:
        """[B, C, H, W] -> [B, (H/p)(W/p), p*p*C] tokens (row-major patches, (p_h, p_w, C) inside)."""
        B, C, H, W = lat.shape
        p = self.config.patch
        return lat.view(B, C, H // p, p, W // p, p).permute(0, 2, 4, 3, 5, 1).reshape(B, (H // p) * (W // p), p * p * C)

    def unpatchify(self, tok: torch.Tensor, H: int, W: int) -> torch.Tensor:
        B = tok.shape[0]
        p, C = self.config.patch, self.config.in_channels
        return tok.view(B, H // p, W // p, p, p, C).permute(0, 5, 1, 3, 2, 4).reshape(B, C, H, W)

    def positions(self, cap_lens: torch.Tensor, Lc: int, hp: int, wp: int):
        """Per distinct caption u: caption token j at (1 + j, 0, 0); image token (h, w) at
        (cap_len_u + 1, h, w).  Returns img_pos [U, hp*wp, 3], cap_pos [Lc, 3]."""
        dev = cap_lens.device
        hh, ww = torch.meshgrid(torch.arange(hp, device=dev), torch.arange(wp, device=dev), indexing="ij")
        img = torch.stack((torch.zeros_like(hh), hh, ww), -1).view(1, hp * wp, 3).repeat(cap_lens.numel(), 1, 1)
        img[..., 0] = cap_lens.view(-1, 1) + 1
        j = torch.arange(Lc, device=dev)
        cap = torch.stack((j + 1, torch.zeros_like(j), torch.zeros_like(j)), -1)
        return img, cap

    def forward(self, lat: torch.Tensor, t: torch.Tensor, cap_feats: torch.Tensor, cap_lens: torch.Tensor,
                enc_index: torch.Tensor, n_rep: int = 1) -> torch.Tensor:
        """lat [n_rep * b, C, H, W] (member-major); t [1] model time in [0, 1] (the step's, shared);
        cap_feats [n_rep * U, Lc, cap_feat_dim] (member-major copies of the U distinct captions, zero
        beyond each); cap_lens [U] the captions' own token counts; enc_index [b] image -> caption.
        Returns the velocity [n_rep * b, C, H, W] (fp32).

        A caption of T tokens is padded to L = T rounded up to seq_multiple with cap_pad_token, and an
        image attends to exactly its N image tokens + its caption's L tokens.  Images are processed in
        groups of equal L (the context refiner per caption group, the main stack per image group), so
        no attention needs a key-padding mask — with one, SDPA leaves the flash kernel for one at half
        its speed.  The groups' images stay member-major, as the population GEMM needs."""
        a = self.config
        Bt, C, H, W = lat.shape
        b, U, Lc = Bt // n_rep, cap_lens.numel(), cap_feats.shape[1]
        hp, wp = H // a.patch, W // a.patch
        N, D, dev = hp * wp, a.dim, lat.device
        m = a.seq_multiple
        if N % m:
            # diffusers pads the image sequence to a multiple of seq_multiple with x_pad_token; those pad
            # tokens take part in attention (and their RoPE positions are unpinned here), so an image
            # whose token count is not a multiple would run a different sequence from the reference
            raise NotImplementedError(f"{hp} x {wp} = {N} image tokens is not a multiple of seq_multiple {m}: "
                                      f"image-token padding (x_pad_token) is not implemented; choose a size "
                                      f"whose patch grid has a multiple of {m} tokens (e.g. 384 or 512 px)")
        real = [int(v) for v in cap_lens.tolist()]
        padl = [-(-r // m) * m for r in real]
        if max(padl) > Lc:
            raise ValueError(f"cap_feats holds {Lc} tokens, a caption needs {max(padl)}")
        ei = [int(v) for v in enc_index.tolist()]
        t_emb = self.t_embedder(t * a.t_scale)                                   # [1, 256] fp32
        x = self.all_x_embedder[f"{a.patch}-1"](self.patchify(lat.to(torch.bfloat16)).contiguous())   # [Bt, N, D]
        cap = self.cap_embedder[1](K.rownorm(cap_feats.to(torch.bfloat16).contiguous(), self.cap_embedder[0].eps,
                                             w=self.cap_embedder[0].weight))     # [n_rep * U, Lc, D]
        # tokens past a caption's own length up to its padded length: cap_pad_token
        valid = torch.arange(Lc, device=dev)[None, :] < cap_lens.to(dev)[:, None]            # [U, Lc]
        cap = torch.where(valid.repeat(n_rep, 1)[..., None], cap, self.cap_pad_token.view(1, 1, -1))
        img_pos, cap_pos = self.positions(torch.tensor(padl, device=dev), Lc, hp, wp)
        ci, si = rope_tables(a, img_pos[enc_index])                              # [b, N, 64]
        for blk in self.noise_refiner:
            blk(x, ci, si, n_rep, None, t_emb)
        fl = self.all_final_layer[f"{a.patch}-1"]
        out = torch.empty(n_rep, b, N, a.patch_dim, device=dev, dtype=torch.bfloat16)
        x4, cap4 = x.view(n_rep, b, N, D), cap.view(n_rep, U, Lc, D)
        for L in sorted(set(padl)):
            ug = [u for u in range(U) if padl[u] == L]
            ig = [j for j in range(b) if padl[ei[j]] == L]
            if not ig:
                continue
            cc, sc = rope_tables(a, cap_pos[:L].expand(len(ug), L, 3))        # [Ug, L, 64]
            cg = cap4[:, ug, :L].reshape(n_rep * len(ug), L, D).contiguous()
            for blk in self.context_refiner:
                blk(cg, cc, sc, n_rep, None)
            loc = [ug.index(ei[j]) for j in ig]
            u = torch.cat((x4[:, ig], cg.view(n_rep, len(ug), L, D)[:, loc]), 2).reshape(n_rep * len(ig), N + L, D)
            cu, su = torch.cat((ci[ig], cc[loc]), 1), torch.cat((si[ig], sc[loc]), 1)
            for blk in self.layers:
                blk(u, cu, su, n_rep, None, t_emb)
            og = fl(u.view(n_rep, len(ig), N + L, D)[:, :, :N].reshape(n_rep * len(ig), N, D), t_emb)
            out[:, ig] = og.view(n_rep, len(ig), N, a.patch_dim)
        return self.unpatchify(out.view(Bt, N, a.patch_dim).float(), H, W)


def zimage_lora_shapes(a: ZImageArch = ZIMAGE_TURBO, r: int = 2, alpha: float = 8.0,
                       targets: Sequence[str] = tuple(ZIMAGE_LORA_TARGETS)) -> List[Tuple[int, ...]]:
    """theta layout (trainable shapes in module.parameters() order) of the LoRA'd transformer, built on
    the meta device: 34 blocks x (to_q, to_k, to_v, w1, w2, w3) + the final layer's linear."""
    with torch.device("meta"):
        model = ZImageTransformer2DModel(a)
        attach_lora(model, r, alpha, targets)
    return [tuple(p.shape) for p in model.parameters() if p.requires_grad]
