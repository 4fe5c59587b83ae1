"""Infinity bitwise autoregressive text-to-image transformer — the host of BASELINE configs[4]'s
perturbed LoRA linears (Infinity-8B, 512 px, LoRA on every block's ffn.fc1), population-batched, bf16.

Reference: `InfinityES` (models/Infinity.py:29-556) builds `Infinity(...)` from the Infinity repo
(models/Infinity.py:19-21, 183-235: shared_aln, rope2d_each_sa_layer=1, rope2d_normalized_by_hw=2,
use_bit_label=1, add_lvl_embeding_only_first_block=0, pad_to_multiplier 128) with the per-variant
depth / width / heads of models/Infinity.py:164-181, wraps it with PEFT on `fc1`
(es_backend.py:798-816, unifed_es.py:472) and samples with `autoregressive_infer_cfg`
(models/Infinity.py:509-537): per-scale CFG from cfg_list, tau_list, top-k / top-p per bit, then the
BSQ-VAE decode.  The Infinity repo is NOT vendored and no weights exist offline, so the transformer,
the multi-scale bit-code accumulation and the VAE decoder here are this build's restatement of the
published design; parity with the Infinity repo is UNPINNED.  What the throughput of configs[4]
depends on — module widths, token counts per scale (2521 tokens per image at 0.25M), CFG doubling,
the KV cache over scales, the LoRA target set (theta D = 1,433,600 at r 2) — follows the reference's
configuration.

MI355X layout: all members of a pass, both CFG halves and all images in ONE batch per scale, rows
member-major ([member][cond | uncond][image][token]) so every linear is one libeggroll population
GEMM (fc1 carries the per-member LoRA; sa.proj / ffn.fc2 fold the gated residual and ca.proj the
residual add into their epilogues); q / k L2 norm + 2-D RoPE in one in-place pass
(eggroll_qk_norm_rope); attention over the per-block KV cache [2, rows, tokens, C] (preallocated for
the whole schedule, read in place) on eggroll_flash_attention; everything text-side (member-independent: no LoRA there) computed once per distinct
prompt.  The reference's generator semantics are kept per micro-batch (es_backend.py:951-1022: every
micro-batch call reseeds with the same seed), so member k's bits equal those of the reference's own
per-member calls given the same logits.
"""
from __future__ import annotations

import math
from dataclasses import dataclass, replace
from typing import Dict, List, Optional, Sequence, Tuple

import torch
import torch.nn.functional as F
from torch import nn

from . import kernels as K
from .flux_vae import FluxVAEDecoder
from .lora import LoRALinear
from .sana import attach_lora
from .var import top_k_top_p_mask_

INFINITY_LORA_TARGETS = ["fc1"]   # unifed_es.py:472


@dataclass
class InfinityArch:
    depth: int = 40
    embed_dim: int = 3584
    num_heads: int = 28
    mlp_ratio: float = 4.0
    block_chunks: int = 8
    text_channels: int = 2048          # flan-t5-xl hidden size (models/Infinity.py:47)
    text_maxlen: int = 512
    codebook_dim: int = 14             # vae_type (models/Infinity.py:131-137)
    spatial_patchify: int = 1          # apply_spatial_patchify: 2x2 VAE pixels per token
    norm_eps: float = 1e-6
    rope_theta: float = 10000.0
    n_levels: int = 15
    vae_widths: Tuple[int, ...] = (160, 320, 640, 640)   # decoder_ch_mult [1, 2, 4, 4] (patchify VAE, f8)

    @property
    def C(self) -> int:
        return self.embed_dim

    @property
    def head_dim(self) -> int:
        return self.embed_dim // self.num_heads

    @property
    def ffn(self) -> int:
        return round(self.embed_dim * self.mlp_ratio)

    @property
    def d_tok(self) -> int:            # bits per token
        return self.codebook_dim * (4 if self.spatial_patchify else 1)

    @property
    def pool_heads(self) -> int:       # TextAttentivePool: head dim 64 above 4096 wide, else 128
        return self.text_channels // (64 if self.embed_dim > 4096 else 128)


# models/Infinity.py:164-181 (depth, embed_dim, num_heads, block_chunks)
INFINITY_VARIANTS: Dict[str, InfinityArch] = {
    "infinity_2b": InfinityArch(depth=32, embed_dim=2048, num_heads=16, block_chunks=8, codebook_dim=32,
                                spatial_patchify=0, vae_widths=(160, 320, 640, 640, 640)),
    "infinity_8b": InfinityArch(),
    "infinity_layer12": InfinityArch(depth=12, embed_dim=768, num_heads=8, block_chunks=4),
    "infinity_layer16": InfinityArch(depth=16, embed_dim=1152, num_heads=12, block_chunks=4),
    "infinity_layer24": InfinityArch(depth=24, embed_dim=1536, num_heads=16, block_chunks=4),
    "infinity_layer32": InfinityArch(depth=32, embed_dim=2080, num_heads=20, block_chunks=4),
    "infinity_layer40": InfinityArch(depth=40, embed_dim=2688, num_heads=24, block_chunks=4),
    "infinity_layer48": InfinityArch(depth=48, embed_dim=3360, num_heads=28, block_chunks=4),
}
INFINITY_8B = INFINITY_VARIANTS["infinity_8b"]

# token-grid side per scale at h/w = 1 for each pn (Infinity's dynamic_resolution templates, final side =
# pixels / 16 with either the f16 VAE or the f8 VAE + 2x2 patchify); UNPINNED restatement
SCALE_SIDES: Dict[str, List[int]] = {
    "0.06M": [1, 2, 4, 6, 8, 12, 16],
    "0.25M": [1, 2, 4, 6, 8, 12, 16, 20, 24, 32],
    "0.60M": [1, 2, 4, 6, 8, 12, 16, 20, 24, 32, 40, 48],
    "1M": [1, 2, 4, 6, 8, 12, 16, 20, 24, 32, 40, 48, 64],
}


def scale_schedule(pn: str) -> List[Tuple[int, int, int]]:
    """models/Infinity.py:86-87: [(1, h, w)] per scale."""
    if pn not in SCALE_SIDES:
        raise ValueError(f"pn={pn!r} unknown (choices {list(SCALE_SIDES)})")
    return [(1, s, s) for s in SCALE_SIDES[pn]]


def _p(*shape, dtype=torch.bfloat16):
    return nn.Parameter(torch.empty(*shape, dtype=dtype), requires_grad=False)


class _Norm(nn.Module):
    def __init__(self, c: int, eps: float, bias: bool):
        super().__init__()
        self.eps = eps
        self.weight = _p(c)
        self.bias = _p(c) if bias else None


class SelfAttention(nn.Module):
    """Cosine attention (q, k L2-normalised per head, logits scaled by exp(min(s_h, log 100))) with
    2-D RoPE, q / v biases, KV cache over the scales."""

    def __init__(self, a: InfinityArch):
        super().__init__()
        C = a.C
        self.heads, self.hd = a.num_heads, a.head_dim
        self.mat_qkv = LoRALinear(C, 3 * C, bias=True, lora=False)   # bias = [q_bias | 0 | v_bias]
        self.scale_mul_1H11 = _p(1, a.num_heads, 1, 1, dtype=torch.float32)
        self.proj = LoRALinear(C, C, bias=True, lora=False)
        self.register_buffer("_ones", torch.ones(128, dtype=torch.bfloat16), persistent=False)


class CrossAttention(nn.Module):
    def __init__(self, a: InfinityArch):
        super().__init__()
        C = a.C
        self.mat_q = LoRALinear(C, C, bias=True, lora=False)
        self.mat_kv = LoRALinear(C, 2 * C, bias=True, lora=False)    # bias = [0 | v_bias]
        self.proj = LoRALinear(C, C, bias=True, lora=False)


class FFN(nn.Module):
    def __init__(self, a: InfinityArch):
        super().__init__()
        self.fc1 = LoRALinear(a.C, a.ffn, bias=True, lora=False)
        self.fc2 = LoRALinear(a.ffn, a.C, bias=True, lora=False)


class CrossAttnBlock(nn.Module):
    """x += gamma1 * sa(LN(x) (1 + scale1) + shift1);  x += ca(LN_affine(x), text);
    x += gamma2 * ffn(LN(x) (1 + scale2) + shift2);  (gamma1, gamma2, scale1, scale2, shift1, shift2) =
    ada_gss + shared_ada_lin(sos) (shared_aln)."""

    def __init__(self, a: InfinityArch):
        super().__init__()
        self.sa = SelfAttention(a)
        self.ca = CrossAttention(a)
        self.ffn = FFN(a)
        self.ca_norm = _Norm(a.C, a.norm_eps, bias=True)
        self.ada_gss = _p(1, 1, 6, a.C, dtype=torch.float32)


class _Chunk(nn.Module):
    def __init__(self, blocks: Sequence[CrossAttnBlock]):
        super().__init__()
        self.module = nn.ModuleList(blocks)


class TextAttentivePool(nn.Module):
    """The start-of-sequence condition: one learned query attending over the (normed) text tokens,
    pool_heads heads; [L, Ct5] -> [C]."""

    def __init__(self, a: InfinityArch):
        super().__init__()
        self.heads = a.pool_heads
        self.query = _p(a.C)
        self.mat_kv = LoRALinear(a.text_channels, 2 * a.C, bias=True, lora=False)
        self.proj = LoRALinear(a.C, a.C, bias=True, lora=False)


class InfinityTransformer(nn.Module):
    def __init__(self, a: InfinityArch = INFINITY_8B):
        super().__init__()
        self.arch = a
        C = a.C
        self.text_norm = _Norm(a.text_channels, a.norm_eps, bias=False)
        self.text_proj_for_sos = TextAttentivePool(a)
        self.text_proj_for_ca = nn.ModuleList([LoRALinear(a.text_channels, C, bias=True, lora=False), nn.GELU("tanh"),
                                               LoRALinear(C, C, bias=True, lora=False)])
        self.cfg_uncond = _p(a.text_maxlen, a.text_channels)
        self.pos_start = _p(1, 1, C)
        self.lvl_embed = _p(a.n_levels, C)
        self.word_embed = LoRALinear(a.d_tok, C, bias=True, lora=False)
        self.shared_ada_lin = nn.ModuleList([nn.SiLU(), LoRALinear(C, 6 * C, bias=True, lora=False)])
        per = a.depth // a.block_chunks
        self.block_chunks = nn.ModuleList([_Chunk([CrossAttnBlock(a) for _ in range(per)])
                                           for _ in range(a.block_chunks)])
        self.head_nm = nn.Module()
        self.head_nm.ada_lin = nn.ModuleList([nn.SiLU(), LoRALinear(C, 2 * C, bias=True, lora=False)])
        self.head = LoRALinear(C, 2 * a.d_tok, bias=True, lora=False)
        # the early scales' plain GEMMs (64 .. 9216 rows at 8B widths) run 1.0-3.9x faster on hipBLASLt's
        # split-K kernels than on the 8-phase / 128-tile kernels (profiles/r07b_small_m_gemm_probe.jsonl)
        for m in self.modules():
            if isinstance(m, LoRALinear):
                m.lib_small_m = 16384

    def blocks(self) -> List[CrossAttnBlock]:
        return [b for ch in self.block_chunks for b in ch.module]

    @torch.no_grad()
    def init_weights(self, seed: int = 0):
        """Synthetic frozen weights: linears N(0, 1/fan_in) (the residual-branch outputs at a third),
        norms 1, q / v biases and AdaLN tables small, cos-attention log-scales log 4 (the Infinity
        init), embeddings N(0, 0.02)."""
        g = torch.Generator(device=self.pos_start.device).manual_seed(seed)

        def rn(p, s):
            p.copy_((torch.randn(p.shape, generator=g, device=p.device, dtype=torch.float32) * s).to(p.dtype))

        for name, p in self.named_parameters():
            if p.requires_grad:
                continue
            if name.endswith("scale_mul_1H11"):
                p.fill_(math.log(4.0))
            elif name.endswith("ada_gss"):
                rn(p, 0.02)
            elif p.ndim >= 2 and not name.endswith(("cfg_uncond", "pos_start", "lvl_embed")):
                std = 1.0 / math.sqrt(p.shape[1])
                if name.endswith(("sa.proj.weight", "ffn.fc2.weight", "ca.proj.weight")):
                    std /= 3.0
                rn(p, std)
            elif p.ndim >= 2 or name.endswith("query"):
                rn(p, 0.02 if not name.endswith("cfg_uncond") else 1.0)
            elif name.endswith("norm.weight"):
                p.fill_(1.0)
            elif name.endswith(".bias") and ("mat_qkv" in name or "mat_kv" in name or "mat_q" in name):
                rn(p, 0.02)
            else:
                p.zero_()
        C = self.arch.C
        for b in self.blocks():   # the k part of [q_bias | 0 | v_bias] and of [0 | v_bias] is structurally zero
            b.sa.mat_qkv.bias[C:2 * C].zero_()
            b.ca.mat_kv.bias[:C].zero_()
        self.text_proj_for_sos.mat_kv.bias[:C].zero_()


def rope2d_tables(a: InfinityArch, h: int, w: int, side: int, device) -> Tuple[torch.Tensor, torch.Tensor]:
    """[h*w, head_dim/2] cos / sin fp32 for a (h, w) token grid, positions normalised to the final
    side (rope2d_normalized_by_hw=2): pairs [0, hd/4) rotate with the row, [hd/4, hd/2) with the column,
    frequencies theta^(-2i / (hd/2)) per axis."""
    half = a.head_dim // 2
    q = half // 2
    inv = 1.0 / (a.rope_theta ** (torch.arange(0, q, dtype=torch.float64, device=device) * 2.0 / half))
    ys = torch.arange(h, dtype=torch.float64, device=device) * (side / h)
    xs = torch.arange(w, dtype=torch.float64, device=device) * (side / w)
    yy, xx = torch.meshgrid(ys, xs, indexing="ij")
    ang = torch.cat((yy.reshape(-1, 1) * inv, xx.reshape(-1, 1) * inv), 1)
    if ang.shape[1] < half:   # odd quarter (head dims not divisible by 4): unrotated tail pairs
        ang = torch.cat((ang, torch.zeros(ang.shape[0], half - ang.shape[1], dtype=ang.dtype, device=device)), 1)
    return torch.cos(ang).float().contiguous(), torch.sin(ang).float().contiguous()


def _rms_rope_torch(x: torch.Tensor, heads: int, hd: int, eps: float, cos: torch.Tensor, sin: torch.Tensor):
    """In place on x [rows, heads*hd] (strided rows): RMS-normalise per head, rotate adjacent pairs by the
    table row = row % tab_rows (the fallback of eggroll_qk_norm_rope for head dims other than 128)."""
    rows = x.shape[0]
    xf = x.float().view(rows, heads, hd)
    xf = xf * torch.rsqrt(xf.pow(2).mean(-1, keepdim=True) + eps)
    ti = torch.arange(rows, device=x.device) % cos.shape[0]
    c, s = cos[ti][:, None, :], sin[ti][:, None, :]
    x0, x1 = xf[..., 0::2], xf[..., 1::2]
    out = torch.stack((x0 * c - x1 * s, x0 * s + x1 * c), -1).reshape(rows, heads * hd)
    x.copy_(out.to(x.dtype))
    return x


def bits_to_codes(bits: torch.Tensor, a: InfinityArch, h: int, w: int) -> torch.Tensor:
    """[N, h*w, d_tok] {0, 1} -> BSQ codes [N, codebook_dim, H', W'] fp32 (+-1 / sqrt(codebook_dim));
    with spatial patchify a token's bits are (channel, dy, dx) of its 2x2 VAE pixels (pixel_shuffle)."""
    N = bits.shape[0]
    c = (bits.float() * 2.0 - 1.0) * (1.0 / math.sqrt(a.codebook_dim))
    c = c.transpose(1, 2).reshape(N, a.d_tok, h, w)
    return F.pixel_shuffle(c, 2) if a.spatial_patchify else c


def codes_to_tokens(z: torch.Tensor, a: InfinityArch) -> torch.Tensor:
    """[N, codebook_dim, H', W'] -> [N, h*w, d_tok] (pixel_unshuffle with spatial patchify)."""
    if a.spatial_patchify:
        z = F.pixel_unshuffle(z, 2)
    N, d, h, w = z.shape
    return z.reshape(N, d, h * w).transpose(1, 2)


def sample_bits(logits: torch.Tensor, gen: torch.Generator, top_k: int, top_p: float) -> torch.Tensor:
    """One reference sampling call (Infinity's sample_with_top_k_top_p_ on [mb, l*d, 2] bit logits with
    top_k clamped to 2): masks in place, one multinomial on `gen`.  logits [mb, l*d, 2] fp32 -> {0,1}."""
    mb, ld, V = logits.shape
    top_k_top_p_mask_(logits, min(int(top_k), V) if top_k > 0 else 0, top_p)
    return torch.multinomial(logits.softmax(dim=-1).view(-1, V), 1, replacement=True, generator=gen).view(mb, ld)


class ChunkedBitSampler:
    """The reference's generation chunks as separate `autoregressive_infer_cfg` calls (es_backend.py's
    micro_batch loop): each chunk call of each member seeds its own generator with g_seed, and that
    generator advances across scales by the chunk's OWN draws.  One generator is replayed per chunk:
    states[c0] is the state chunk c0's generator holds before the current scale.  Members start every
    chunk from the same state (each member's calls are independent, unifed_es.py:159-163); a smaller
    last chunk (B % micro_batch != 0) keeps its own state sequence."""

    def __init__(self, gen: torch.Generator, B: int, mb: int):
        self.gen, self.B, self.mb = gen, int(B), int(mb)
        st = gen.get_state()
        self.states = {c0: st for c0 in range(0, self.B, self.mb)}

    def sample(self, lg: torch.Tensor, top_k: int, top_p: float) -> torch.Tensor:
        """lg [n, B, l*d, 2] CFG'd logits of one scale -> bits [n, B, l*d] (long)."""
        n = lg.shape[0]
        bits = torch.empty(lg.shape[:3], dtype=torch.long, device=lg.device)
        for c0, pre in self.states.items():
            c1 = min(self.B, c0 + self.mb)
            post = None
            for k in range(n):
                self.gen.set_state(pre)
                bits[k, c0:c1] = sample_bits(lg[k, c0:c1], self.gen, top_k, top_p)
                post = self.gen.get_state()
            self.states[c0] = post
        return bits


class InfinityPopulationInfer:
    """`autoregressive_infer_cfg` (models/Infinity.py:509-537) for n members at once."""

    def __init__(self, tr: InfinityTransformer, vae: FluxVAEDecoder):
        self.tr, self.vae = tr, vae
        self.use_kernel = True    # eggroll_qk_norm_rope + eggroll_flash_attention at head dim 128 (False: torch forms)

    # ---- text side (member-independent) ------------------------------------------------
    def _text(self, kv_list: Sequence[torch.Tensor], lens: Sequence[int]):
        """Distinct prompts -> cond + uncond rows [2U, ...]: per-row key bias [2U, Lt], sos [2U, C] fp32,
        ca tokens [2U, Lt, C] bf16.  The unconditional text of a prompt of length L is cfg_uncond[:L]."""
        tr, a = self.tr, self.tr.arch
        dev = tr.pos_start.device
        U = len(kv_list)
        Lt = max(int(v) for v in lens)
        if Lt > a.text_maxlen:
            raise ValueError(f"text of {Lt} tokens > text_maxlen {a.text_maxlen}")
        t = torch.zeros(2 * U, Lt, a.text_channels, device=dev, dtype=torch.float32)
        for u, (kv, L) in enumerate(zip(kv_list, lens)):
            t[u, :L] = kv[:L].to(dev, torch.float32)
            t[U + u, :L] = tr.cfg_uncond[:L].float()
        valid = torch.arange(Lt, device=dev)[None, :] < torch.tensor(list(lens) * 2, device=dev)[:, None]
        bias = torch.zeros(2 * U, Lt, device=dev).masked_fill_(~valid, float("-inf"))
        tn = tr.text_norm
        t = t * torch.rsqrt(t.pow(2).mean(-1, keepdim=True) + tn.eps) * tn.weight.float()
        # sos: attentive pool (fp32; 2U rows)
        pool = tr.text_proj_for_sos
        H = pool.heads
        kv = pool.mat_kv.forward_fp32(t).view(2 * U, Lt, 2, H, a.C // H)
        q = pool.query.float().view(1, H, 1, a.C // H).expand(2 * U, H, 1, a.C // H)
        o = F.scaled_dot_product_attention(q, kv[:, :, 0].transpose(1, 2), kv[:, :, 1].transpose(1, 2),
                                           attn_mask=bias[:, None, None, :])
        sos = pool.proj.forward_fp32(o.reshape(2 * U, a.C))
        ca = tr.text_proj_for_ca
        cat = ca[2](F.gelu(ca[0](t.to(torch.bfloat16)), approximate="tanh"))          # [2U, Lt, C]
        return bias, sos, cat

    def _qscale(self, sa: SelfAttention, H: int, hd: int) -> torch.Tensor:
        """exp(min(s_h, log 100)) / hd per head, bf16-rounded (the factor torch's bf16 multiply applies),
        held as fp32; cached per module (the log-scales are frozen)."""
        key = (sa.scale_mul_1H11._version, sa.scale_mul_1H11.data_ptr())
        if getattr(sa, "_qs_key", None) != key:
            qs = sa.scale_mul_1H11.view(H).clamp(max=math.log(100.0)).exp() / hd
            sa._qs, sa._qs_key = qs.to(torch.bfloat16).float().contiguous(), key
        return sa._qs

    # ---- one scale step through the blocks ----------------------------------------------
    def _block(self, blk: CrossAttnBlock, x, l, cur, kv, mod32, mod16, cak, cav, cabias, cos, sin):
        a = self.tr.arch
        C, H, hd = a.C, a.num_heads, a.head_dim
        N2 = x.shape[0] // l
        sa = blk.sa
        h = K.rownorm(x, a.norm_eps, layer=True, mscale=mod32[:, 2], mshift=mod32[:, 4], rows_per_group=l)
        qkv = sa.mat_qkv(h)                                                             # [N2*l, 3C]
        q2, k2 = qkv[:, :C], qkv[:, C:2 * C]
        # RMS-normalised rows have norm sqrt(hd): logits = exp(s_h) cos(q, k) = (q * exp(s_h) / hd) . k
        if self.use_kernel and hd == 128:
            # q: norm + RoPE + the per-head scale in place; k: norm + RoPE written straight into the cache
            # slice, the values copied alongside (no separate scale / copy passes)
            K.qk_norm_rope_kv(q2, sa._ones, 1e-12, cos, sin, H, hscale=self._qscale(sa, H, hd))
            K.qk_norm_rope_kv(k2, sa._ones, 1e-12, cos, sin, H, out=kv[0], rows_per_seq=l, row0=cur,
                              vin=qkv[:, 2 * C:], vout=kv[1])
            q = qkv.view(N2, l, 3, H, hd)[:, :, 0]
        else:
            _rms_rope_torch(q2, H, hd, 1e-12, cos, sin)
            _rms_rope_torch(k2, H, hd, 1e-12, cos, sin)
            q = qkv.view(N2, l, 3, H, hd)[:, :, 0] * self._qscale(sa, H, hd).to(torch.bfloat16).view(1, 1, H, 1)
            kv[0, :, cur:cur + l] = k2.view(N2, l, C)
            kv[1, :, cur:cur + l] = qkv.view(N2, l, 3, C)[:, :, 2]
        ks = kv[0, :, :cur + l].view(N2, cur + l, H, hd)
        vs = kv[1, :, :cur + l].view(N2, cur + l, H, hd)
        if self.use_kernel and hd == 128:     # eggroll_flash_attention reads q from qkv and the cache in place
            o = K.flash_attention(q, ks, vs, 1.0).view(N2 * l, C)
        else:
            o = F.scaled_dot_product_attention(q.transpose(1, 2), ks.transpose(1, 2), vs.transpose(1, 2), scale=1.0)
            o = o.transpose(1, 2).reshape(N2 * l, C)
        sa.proj(o, epi="gated", res=x, gate=mod16[:, 0], rows_per_group=l)
        # cross-attention to the text (keys: this row's prompt, cond or uncond)
        cn = blk.ca_norm
        h = K.rownorm(x, a.norm_eps, layer=True, w=cn.weight, b=cn.bias)
        if isinstance(cak, tuple):   # eggroll_cross_attention: k / v read in place from the distinct text rows
            kvo, drow_i, bias16 = cak
            Lt = bias16.shape[1]
            o = K.cross_attention(blk.ca.mat_q(h), kvo[:, :C], kvo[:, C:], N2, l, H, hd, Lt, hd ** -0.5,
                                  bias=bias16, enc_index=drow_i)
        else:
            q = blk.ca.mat_q(h).view(N2, l, H, hd).transpose(1, 2)
            o = F.scaled_dot_product_attention(q, cak, cav, attn_mask=cabias, scale=hd ** -0.5)
            o = o.transpose(1, 2).reshape(N2 * l, C)
        blk.ca.proj(o, epi="res", res=x)
        h = K.rownorm(x, a.norm_eps, layer=True, mscale=mod32[:, 3], mshift=mod32[:, 5], rows_per_group=l)
        f = blk.ffn.fc1(h, epi="gelu")          # GELU(tanh) in the GEMM epilogue where it applies
        blk.ffn.fc2(f, epi="gated", res=x, gate=mod16[:, 1], rows_per_group=l)

    @torch.no_grad()
    def run(self, kv_list: Sequence[torch.Tensor], lens: Sequence[int], prompt_index: torch.Tensor, n: int,
            schedule: Sequence[Tuple[int, int, int]], g_seed: int, cfg_list: Sequence[float],
            tau_list: Sequence[float], top_k: int, top_p: float, micro_batch: int = 0,
            force_bits: Optional[List[torch.Tensor]] = None, keep_logits: bool = False):
        """kv_list / lens: the DISTINCT prompts' T5 features; prompt_index [B] image -> distinct prompt
        (shared by all members); n members (population context already set, or n = 1 with the model's
        own LoRA).  micro_batch: the reference's generation chunk (es_backend.py:951-1022: every chunk
        call reseeds its generator with g_seed); 0 = one call for all B.  force_bits: optional per-scale
        [n*B, l, d_tok] bits replacing the sampled ones (teacher forcing, parity tests).
        Returns (summed codes [n*B, codebook_dim, H', W'] fp32, per-scale bits, per-scale CFG logits)."""
        tr, a = self.tr, self.tr.arch
        C, H, hd = a.C, a.num_heads, a.head_dim
        dev = tr.pos_start.device
        B = int(prompt_index.numel())
        U = len(kv_list)
        N2 = 2 * B * n
        pidx = prompt_index.to(dev).long()
        # row s = ((k * 2 + half) * B + j) -> distinct text row half * U + pidx[j]
        drow = torch.cat((pidx, pidx + U)).repeat(n)                                        # [N2]
        bias, sos, cat = self._text(kv_list, lens)
        Lt = cat.shape[1]
        shared = tr.shared_ada_lin[1].forward_fp32(F.silu(sos))                             # [2U, 6C]
        ada_h = tr.head_nm.ada_lin[1].forward_fp32(F.silu(sos))[drow]                       # [N2, 2C]
        cabias = bias[drow][:, None, None, :].to(torch.bfloat16)
        blocks = tr.blocks()
        per_chunk = len(blocks) // len(tr.block_chunks)
        ltot = sum(h * w for _, h, w in schedule)
        side = schedule[-1][1]
        vside = side * (2 if a.spatial_patchify else 1)
        # per-block constants: modulation rows (fp32 for the norms, bf16 gates for the epilogues) and the
        # text keys / values gathered per row
        mods, cas = [], []
        # text cross-attention on eggroll_cross_attention (head dim 128 stages <= 256 keys): each row's k / v
        # are its distinct text row's, addressed through enc_index = drow, the mask an additive bf16 bias
        xa_kernel = self.use_kernel and hd == 128 and Lt <= 256
        if xa_kernel:
            drow_i, bias16 = drow.to(torch.int32).contiguous(), bias.to(torch.bfloat16).contiguous()
        for blk in blocks:
            m32 = (blk.ada_gss.view(1, 6, C) + shared.view(-1, 6, C))[drow].contiguous()    # [N2, 6, C]
            m16 = m32[:, :2].to(torch.bfloat16).contiguous()
            mods.append((m32, m16))
            if xa_kernel:
                cas.append(((blk.ca.mat_kv(cat.reshape(2 * U * Lt, -1)), drow_i, bias16), None))
                continue
            kvt = blk.ca.mat_kv(cat).view(2 * U, Lt, 2, H, hd)
            cas.append((kvt[:, :, 0][drow].transpose(1, 2), kvt[:, :, 1][drow].transpose(1, 2)))
        caches = [torch.empty((2, N2, ltot, C), dtype=torch.bfloat16, device=dev) for _ in blocks]
        x = (sos[drow] + tr.pos_start.float().view(1, C)).to(torch.bfloat16).contiguous()   # [N2 * 1, C]
        summed = torch.zeros((n * B, a.codebook_dim, vside, vside), dtype=torch.float32, device=dev)
        mb = B if micro_batch <= 0 or micro_batch >= B else int(micro_batch)
        sampler = ChunkedBitSampler(torch.Generator(device=dev).manual_seed(int(g_seed)), B, mb)
        bits_all, logits_all = [], []
        cur = 0
        for si, (_, h, w) in enumerate(schedule):
            l = h * w
            cos, sin = rope2d_tables(a, h, w, side, dev)
            lvl = tr.lvl_embed[si].view(1, C)
            for bi, blk in enumerate(blocks):
                if bi % per_chunk == 0:       # add_lvl_embeding_only_first_block = 0: before every chunk
                    x.add_(lvl)
                m32, m16 = mods[bi]
                self._block(blk, x, l, cur, caches[bi], m32, m16, cas[bi][0], cas[bi][1], cabias, cos, sin)
            cur += l
            hn = K.rownorm(x, a.norm_eps, layer=True, mscale=ada_h[:, :C], mshift=ada_h[:, C:], rows_per_group=l)
            lg = tr.head(hn).float().view(n, 2, B, l * a.d_tok, 2) / float(tau_list[si])
            cfg = float(cfg_list[si])
            lg = cfg * lg[:, 0] + (1.0 - cfg) * lg[:, 1]                                   # [n, B, l*d, 2]
            if keep_logits:
                logits_all.append(lg.clone())
            if force_bits is not None:
                bits = force_bits[si].to(dev).view(n, B, l * a.d_tok).long()
            else:
                bits = sampler.sample(lg, top_k, top_p)
            bits = bits.view(n * B, l, a.d_tok)
            bits_all.append(bits)
            codes = bits_to_codes(bits, a, h, w)
            if si != len(schedule) - 1:
                summed.add_(F.interpolate(codes, size=(vside, vside), mode="bilinear", align_corners=False))
                _, h2, w2 = schedule[si + 1]
                vh = h2 * (2 if a.spatial_patchify else 1)
                nxt = codes_to_tokens(F.interpolate(summed, size=(vh, vh), mode="area"), a)       # [nB, l', d]
                e = tr.word_embed.forward_fp32(nxt)                                            # [nB, l', C]
                x = e.view(n, 1, B, h2 * w2, C).expand(n, 2, B, h2 * w2, C).to(torch.bfloat16).reshape(-1, C)
                x = x.contiguous()
            else:
                summed.add_(codes)
        return summed, bits_all, logits_all


def infinity_lora_shapes_from_model(a: InfinityArch = INFINITY_8B, r: int = 2, alpha: float = 8.0,
                                    targets: Sequence[str] = tuple(INFINITY_LORA_TARGETS)) -> List[Tuple[int, ...]]:
    """theta layout of the LoRA'd transformer (trainable shapes in parameter order), meta device."""
    with torch.device("meta"):
        m = InfinityTransformer(a)
        attach_lora(m, r, alpha, targets)
    return [tuple(p.shape) for p in m.parameters() if p.requires_grad]


def infinity_vae(a: InfinityArch) -> FluxVAEDecoder:
    """The BSQ-VAE decoder: codebook_dim latent channels, LDM-style up path (2 + 1 ResnetBlocks per
    level, mid attention), 8x (patchify VAE, ch_mult [1, 2, 4, 4]) or 16x upsampling."""
    return FluxVAEDecoder(latent_channels=a.codebook_dim, widths=a.vae_widths, layers=2,
                          scaling_factor=1.0, shift_factor=0.0)


def arch_for(model_type: str, vae_type: int, apply_spatial_patchify: int, text_channels: int = 2048) -> InfinityArch:
    """models/Infinity.py:131-181: the variant's transformer + the VAE the vae_type / patchify imply."""
    if model_type not in INFINITY_VARIANTS:
        raise ValueError(f"Unknown model_type={model_type}")
    if vae_type not in (14, 16, 18, 20, 24, 32, 64):
        raise ValueError(f"vae_type={vae_type} not supported")
    widths = (160, 320, 640, 640) if apply_spatial_patchify else (160, 320, 640, 640, 640)
    return replace(INFINITY_VARIANTS[model_type], codebook_dim=int(vae_type), spatial_patchify=int(apply_spatial_patchify),
                   text_channels=int(text_channels), vae_widths=widths)
