"""VAR class-conditional generator (BASELINE configs[0]) — population-batched on the ES hot path.

Reference: `models/VAR.py:27-334` (`VARClassGenerator`, the ES wrapper) on the reference's own
`VAR_models` package: `var.py:21-190` (VAR, `autoregressive_infer_cfg`), `basic_var.py:33-174`
(FFN, SelfAttention with KV cache, AdaLNSelfAttn, AdaLNBeforeHead), `quant.py:15-243`
(VectorQuantizer2 next-scale input, Phi / PhiPartiallyShared), `vqvae.py:16-63` (`fhat_to_img`),
`basic_vae.py:40-226` (Decoder), `helpers.py:6-19` (top-k / top-p sampling).  LoRA is attached by
PEFT suffix matching of `mat_qkv, proj, fc1, fc2, ada_lin.1, head_nm.ada_lin.1, head`
(es_backend.py:334-341, unifed_es.py:403-406).

What is different from the reference, by design:
  * every member of the local population runs in ONE forward per scale: sequences are stacked
    member-major as [member][cond B | uncond B] (the reference's CFG doubling, var.py:151), and every
    PEFT target is an `eggroll_lora_linear_pop` (LoRA'd GEMM per member, rows_per_member = 2B*l);
  * the AdaLN modulations depend only on the class condition, so they are computed once per
    generation instead of once per scale (same values: var.py:165 recomputes the same function);
  * the KV cache is preallocated [seq, heads, L, 64] per block and written in place (var: cat);
  * transformer activations are bf16 (MFMA), the reference runs fp16 autocast on CUDA
    (models/VAR.py:298-304); the token-map / f_hat path (codebook, bicubic / area resampling, Phi)
    stays fp32 as in the reference; the VQVAE decoder runs bf16 channels-last convolutions;
  * sampling: each member keeps its own device Generator seeded with g_seed (the reference seeds
    `self.rng` once per member's generate call, var.py:143-144), so member k's multinomial draws
    consume exactly the stream the reference's k-th generate call would.
State-dict keys are the reference's (`var_d16.pth` / `vae_ch160v4096z32.pth` load with
`load_reference_state`), so a real checkpoint drops in; without one, weights are synthetic.
"""
from __future__ import annotations

import math
from dataclasses import dataclass
from typing import Dict, Iterable, List, Optional, Sequence, Tuple

import numpy as np
import torch
import torch.nn.functional as F
from torch import nn

from . import kernels as K
from .lora import LoRALinear, PopulationContext, set_population

VAR_LORA_TARGETS = ["mat_qkv", "proj", "fc1", "fc2", "ada_lin.1", "head_nm.ada_lin.1", "head"]  # unifed_es.py:406


@dataclass(frozen=True)
class VARArch:
    """build_vae_var (VAR_models/__init__.py:9-39) hyper-parameters: heads = depth, width = 64 depth."""
    depth: int = 16
    patch_nums: Tuple[int, ...] = (1, 2, 3, 4, 5, 6, 8, 10, 13, 16)
    vocab_size: int = 4096
    Cvae: int = 32
    num_classes: int = 1000
    mlp_ratio: float = 4.0
    norm_eps: float = 1e-6
    vae_ch: int = 160
    vae_ch_mult: Tuple[int, ...] = (1, 1, 2, 2, 4)
    vae_num_res_blocks: int = 2
    share_quant_resi: int = 4
    quant_resi: float = 0.5

    @property
    def C(self) -> int:
        return 64 * self.depth

    @property
    def heads(self) -> int:
        return self.depth

    @property
    def L(self) -> int:
        return sum(p * p for p in self.patch_nums)


VAR_D16 = VARArch()


# ---------------------------------------------------------------------------------------
# transformer (VAR_models/var.py, basic_var.py) — parameter names = the reference's
# ---------------------------------------------------------------------------------------


class VARSelfAttention(nn.Module):
    """basic_var.py:58-125 with attn_l2_norm=True (build_vae_var default): q, k L2-normalised,
    q scaled by exp(min(scale_mul, log 100)) per head, softmax scale 1."""

    def __init__(self, C: int, heads: int):
        super().__init__()
        self.heads, self.head_dim = heads, C // heads
        self.scale_mul_1H11 = nn.Parameter(torch.full((1, heads, 1, 1), 4.0).log(), requires_grad=False)
        self.max_scale_mul = math.log(100.0)
        self.mat_qkv = LoRALinear(C, 3 * C, bias=False, lora=False)
        self.q_bias = nn.Parameter(torch.zeros(C), requires_grad=False)
        self.v_bias = nn.Parameter(torch.zeros(C), requires_grad=False)
        self.proj = LoRALinear(C, C, lora=False)

    def refresh(self):
        """The effective qkv bias cat(q_bias, 0, v_bias) (basic_var.py:93) in bf16 for the GEMM
        epilogue, and the per-head q multiplier exp(min(scale_mul, log 100))."""
        self.qkv_bias = torch.cat((self.q_bias, torch.zeros_like(self.q_bias), self.v_bias)).to(torch.bfloat16)
        self.q_mul = self.scale_mul_1H11.float().clamp_max(self.max_scale_mul).exp()   # [1, H, 1, 1]

    def qkv(self, h: torch.Tensor) -> torch.Tensor:
        """basic_var.py:93 calls F.linear(weight=self.mat_qkv.weight, ...) instead of the module: under
        PEFT, `.weight` of the wrapped layer is the BASE weight, so the reference's mat_qkv LoRA
        parameters sit in theta (they are perturbed and updated) but never reach the output.  The
        build reproduces that: the plain GEMM, no LoRA term (pinned by g11)."""
        return K.lora_linear_pop(h.contiguous(), self.mat_qkv.weight, self.qkv_bias, None, 0, 0, 0, 0.0, h.shape[0])


class VARFFN(nn.Module):
    def __init__(self, C: int, hidden: int):
        super().__init__()
        self.fc1 = LoRALinear(C, hidden, lora=False)
        self.fc2 = LoRALinear(hidden, C, lora=False)


class VARBlock(nn.Module):
    """AdaLNSelfAttn (basic_var.py:128-162), shared_aln=False."""

    def __init__(self, C: int, heads: int, mlp_ratio: float):
        super().__init__()
        self.attn = VARSelfAttention(C, heads)
        self.ffn = VARFFN(C, round(C * mlp_ratio))
        self.ada_lin = nn.Sequential(nn.SiLU(), LoRALinear(C, 6 * C, lora=False))


class AdaLNBeforeHead(nn.Module):
    def __init__(self, C: int):
        super().__init__()
        self.ada_lin = nn.Sequential(nn.SiLU(), LoRALinear(C, 2 * C, lora=False))


class VARTransformer(nn.Module):
    """VAR (var.py:21-116): the LoRA target.  Registration order = the reference's, so the trainable
    parameters come out in the reference theta order (utills.py:141-152)."""

    def __init__(self, a: VARArch = VAR_D16):
        super().__init__()
        self.arch = a
        C = a.C
        self.word_embed = nn.Linear(a.Cvae, C)
        self.class_emb = nn.Embedding(a.num_classes + 1, C)
        self.pos_start = nn.Parameter(torch.zeros(1, a.patch_nums[0] ** 2, C))
        self.pos_1LC = nn.Parameter(torch.zeros(1, a.L, C))
        self.lvl_embed = nn.Embedding(len(a.patch_nums), C)
        self.blocks = nn.ModuleList([VARBlock(C, a.heads, a.mlp_ratio) for _ in range(a.depth)])
        self.head_nm = AdaLNBeforeHead(C)
        self.head = LoRALinear(C, a.vocab_size, lora=False)
        for p in self.parameters():
            p.requires_grad_(False)
        lvl = torch.cat([torch.full((pn * pn,), i) for i, pn in enumerate(a.patch_nums)])
        self.register_buffer("lvl_1L", lvl.view(1, -1), persistent=False)

    @torch.no_grad()
    def init_weights(self, seed: int = 0):
        """Synthetic weights when no checkpoint is present: the reference's init_weights recipe
        (var.py:236-286 with build_vae_var's init_adaln 0.5, init_adaln_gamma 1e-5, init_head 0.02,
        init_std sqrt(1/3C)) drawn from a seeded generator — except the AdaLN gamma rows, scaled up
        to 0.5 like the others so a synthetic model's blocks are not near-identities."""
        a, C = self.arch, self.arch.C
        g = torch.Generator(device=self.pos_1LC.device).manual_seed(seed)
        std = math.sqrt(1.0 / C / 3.0)

        def tn(p, s):
            p.copy_(torch.randn(p.shape, generator=g, device=p.device).clamp_(-2, 2).mul_(s).to(p.dtype))

        for mod in self.modules():
            if isinstance(mod, (nn.Linear, LoRALinear)):
                tn(mod.weight, std)
                if isinstance(mod.bias, nn.Parameter):
                    mod.bias.zero_()
            elif isinstance(mod, nn.Embedding):
                tn(mod.weight, std)
        tn(self.pos_start, std)
        tn(self.pos_1LC, std)
        self.head.weight.mul_(0.02 * 25)          # init_head (x25: synthetic logits need spread to sample)
        self.head_nm.ada_lin[1].weight.mul_(0.5)
        for blk in self.blocks:
            blk.attn.proj.weight.div_(math.sqrt(2 * a.depth))
            blk.ffn.fc2.weight.div_(math.sqrt(2 * a.depth))
            blk.ada_lin[1].weight.mul_(0.5)
        self.refresh()

    def refresh(self):
        for blk in self.blocks:
            blk.attn.refresh()


# ---------------------------------------------------------------------------------------
# VQVAE decode side (quant.py, vqvae.py, basic_vae.py)
# ---------------------------------------------------------------------------------------


class DConv2d(nn.Conv2d):
    """nn.Conv2d (same parameters) whose small-map launches run as an explicit im2col GEMM.  The
    reference asks for deterministic convolutions (models/VAR.py:80-81); on this stack MIOpen's bf16
    solvers for the 16x16 maps at 640 channels differ run to run (tools/var_det_probe.py) and its
    deterministic mode finds no algorithm for them, so maps of <= 32x32 pixels take the GEMM path."""

    def forward(self, x):
        N, C, H, W = x.shape
        if H * W > 1024:
            return super().forward(x)
        wf = getattr(self, "_wflat", None)
        if wf is None or wf.dtype != self.weight.dtype:
            wf = self._wflat = self.weight.detach().contiguous().view(self.out_channels, -1)
        if self.kernel_size == (1, 1):
            y = F.linear(x.permute(0, 2, 3, 1).reshape(-1, C), wf, self.bias)
            return y.view(N, H, W, -1).permute(0, 3, 1, 2)
        cols = F.unfold(x, self.kernel_size, padding=self.padding)             # [N, C*k*k, HW]
        y = torch.matmul(wf, cols)
        if self.bias is not None:
            y = y + self.bias.view(1, -1, 1)
        return y.view(N, self.out_channels, H, W)


def _norm(c: int) -> nn.GroupNorm:
    return nn.GroupNorm(32, c, eps=1e-6, affine=True)


class ResnetBlock(nn.Module):
    """basic_vae.py:40-60."""

    def __init__(self, cin: int, cout: int):
        super().__init__()
        self.norm1 = _norm(cin)
        self.conv1 = DConv2d(cin, cout, 3, 1, 1)
        self.norm2 = _norm(cout)
        self.conv2 = DConv2d(cout, cout, 3, 1, 1)
        self.nin_shortcut = DConv2d(cin, cout, 1) if cin != cout else nn.Identity()

    def forward(self, x):
        h = self.conv1(F.silu(self.norm1(x)))
        h = self.conv2(F.silu(self.norm2(h)))
        return self.nin_shortcut(x) + h


class AttnBlock(nn.Module):
    """basic_vae.py:63-92: single-head attention over the H*W pixels, scale C^-1/2."""

    def __init__(self, c: int):
        super().__init__()
        self.C = c
        self.norm = _norm(c)
        self.qkv = DConv2d(c, 3 * c, 1)
        self.proj_out = DConv2d(c, c, 1)

    def forward(self, x):
        B, C, H, W = x.shape
        qkv = self.qkv(self.norm(x)).reshape(B, 3, C, H * W)
        q, k, v = (qkv[:, i].transpose(1, 2)[:, None] for i in range(3))      # [B, 1, HW, C]
        h = F.scaled_dot_product_attention(q, k, v, scale=C ** -0.5)[:, 0]    # [B, HW, C]
        return x + self.proj_out(h.transpose(1, 2).reshape(B, C, H, W))


class Upsample2x(nn.Module):
    def __init__(self, c: int):
        super().__init__()
        self.conv = DConv2d(c, c, 3, 1, 1)

    def forward(self, x):
        return self.conv(F.interpolate(x, scale_factor=2, mode="nearest"))


class VQDecoder(nn.Module):
    """basic_vae.py:163-226 (using_sa, using_mid_sa)."""

    def __init__(self, ch: int, ch_mult: Sequence[int], num_res_blocks: int, z_channels: int):
        super().__init__()
        n = len(ch_mult)
        block_in = ch * ch_mult[-1]
        self.conv_in = DConv2d(z_channels, block_in, 3, 1, 1)
        self.mid = nn.Module()
        self.mid.block_1 = ResnetBlock(block_in, block_in)
        self.mid.attn_1 = AttnBlock(block_in)
        self.mid.block_2 = ResnetBlock(block_in, block_in)
        self.up = nn.ModuleList()
        for i_level in reversed(range(n)):
            up = nn.Module()
            up.block, up.attn = nn.ModuleList(), nn.ModuleList()
            block_out = ch * ch_mult[i_level]
            for _ in range(num_res_blocks + 1):
                up.block.append(ResnetBlock(block_in, block_out))
                block_in = block_out
                if i_level == n - 1:
                    up.attn.append(AttnBlock(block_in))
            if i_level != 0:
                up.upsample = Upsample2x(block_in)
            self.up.insert(0, up)
        self.norm_out = _norm(block_in)
        self.conv_out = DConv2d(block_in, 3, 3, 1, 1)
        self.n, self.nrb = n, num_res_blocks

    def forward(self, z):
        h = self.mid.block_2(self.mid.attn_1(self.mid.block_1(self.conv_in(z))))
        for i_level in reversed(range(self.n)):
            up = self.up[i_level]
            for i_block in range(self.nrb + 1):
                h = up.block[i_block](h)
                if len(up.attn) > 0:
                    h = up.attn[i_block](h)
            if i_level != 0:
                h = up.upsample(h)
        return self.conv_out(F.silu(self.norm_out(h)))


class _Quantize(nn.Module):
    """The inference half of VectorQuantizer2 (quant.py:15-197): codebook + partially shared Phi."""

    def __init__(self, a: VARArch):
        super().__init__()
        self.embedding = nn.Embedding(a.vocab_size, a.Cvae)
        self.quant_resi = nn.Module()
        self.quant_resi.qresi_ls = nn.ModuleList([nn.Conv2d(a.Cvae, a.Cvae, 3, 1, 1) for _ in range(a.share_quant_resi)])
        K_ = a.share_quant_resi
        self.ticks = (np.linspace(1 / 3 / K_, 1 - 1 / 3 / K_, K_) if K_ == 4 else np.linspace(1 / 2 / K_, 1 - 1 / 2 / K_, K_))
        self.resi = abs(a.quant_resi)

    def phi(self, at: float, h: torch.Tensor) -> torch.Tensor:
        """quant.py:199-226: Phi(h) = (1 - r) h + r conv3x3(h), the conv picked by the nearest tick."""
        conv = self.quant_resi.qresi_ls[int(np.argmin(np.abs(self.ticks - at)))]
        y = F.conv2d(h, conv.weight.float(), conv.bias.float(), padding=1)
        return h.mul(1 - self.resi) + y.mul_(self.resi)


class VQVAEDecode(nn.Module):
    """VQVAE (vqvae.py:16-63) minus the encoder: keys quantize.*, post_quant_conv.*, decoder.*."""

    def __init__(self, a: VARArch):
        super().__init__()
        self.arch = a
        self.quantize = _Quantize(a)
        self.post_quant_conv = nn.Conv2d(a.Cvae, a.Cvae, 3, 1, 1)
        self.decoder = VQDecoder(a.vae_ch, a.vae_ch_mult, a.vae_num_res_blocks, a.Cvae)
        for p in self.parameters():
            p.requires_grad_(False)

    @torch.no_grad()
    def init_weights(self, seed: int = 0):
        """Synthetic VQVAE (no checkpoint): N(0, 1/fan_in) convs, unit norms, N(0,1) codebook."""
        g = torch.Generator(device=self.post_quant_conv.weight.device).manual_seed(seed)
        for name, p in self.named_parameters():
            if name.endswith("embedding.weight"):
                p.copy_(torch.randn(p.shape, generator=g, device=p.device))
            elif p.dim() > 1:
                p.copy_(torch.randn(p.shape, generator=g, device=p.device) / math.sqrt(p[0].numel()))
            elif "norm" in name and name.endswith("weight"):
                p.fill_(1.0)
            else:
                p.zero_()

    def next_autoregressive_input(self, si: int, SN: int, f_hat: torch.Tensor, h_BChw: torch.Tensor):
        """quant.py:187-196 (in place on f_hat, fp32)."""
        HW = self.arch.patch_nums[-1]
        if si != SN - 1:
            f_hat.add_(self.quantize.phi(si / (SN - 1), F.interpolate(h_BChw, size=(HW, HW), mode="bicubic")))
            pn = self.arch.patch_nums[si + 1]
            return f_hat, F.interpolate(f_hat, size=(pn, pn), mode="area")
        f_hat.add_(self.quantize.phi(si / (SN - 1), h_BChw))
        return f_hat, f_hat

    def fhat_to_img(self, f_hat: torch.Tensor, chunk: int = 16) -> torch.Tensor:
        """vqvae.py:62-63: decoder(post_quant_conv(f_hat)).clamp(-1, 1), bf16 channels-last."""
        z = F.conv2d(f_hat, self.post_quant_conv.weight.float(), self.post_quant_conv.bias.float(), padding=1)
        outs = []
        for s in range(0, z.shape[0], chunk):
            zc = z[s:s + chunk].to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
            outs.append(self.decoder(zc).clamp_(-1, 1))
        return torch.cat(outs)


# ---------------------------------------------------------------------------------------
# sampling (helpers.py:6-19)
# ---------------------------------------------------------------------------------------


def top_k_top_p_mask_(logits: torch.Tensor, top_k: int = 0, top_p: float = 0.0) -> torch.Tensor:
    """helpers.py:8-15 over the last dim, in place (row-wise: identical for any batch stacking)."""
    if top_k > 0:
        kth = logits.topk(top_k, largest=True, sorted=False, dim=-1)[0].amin(dim=-1, keepdim=True)
        logits.masked_fill_(logits < kth, -torch.inf)
    if top_p > 0:
        sorted_logits, sorted_idx = logits.sort(dim=-1, descending=False)
        rm = sorted_logits.softmax(dim=-1).cumsum_(dim=-1) <= (1 - top_p)
        rm[..., -1:] = False
        logits.masked_fill_(rm.scatter(sorted_idx.ndim - 1, sorted_idx, rm), -torch.inf)
    return logits


def sample_with_top_k_top_p_(logits_BlV: torch.Tensor, top_k: int = 0, top_p: float = 0.0, rng=None,
                             num_samples: int = 1) -> torch.Tensor:
    """helpers.py:6-19: returns idx [B, l, num_samples]."""
    B, l, V = logits_BlV.shape
    top_k_top_p_mask_(logits_BlV, top_k, top_p)
    replacement = num_samples >= 0
    num_samples = abs(num_samples)
    return torch.multinomial(logits_BlV.softmax(dim=-1).view(-1, V), num_samples=num_samples,
                             replacement=replacement, generator=rng).view(B, l, num_samples)


def sample_population(logits: torch.Tensor, gens: Sequence[torch.Generator], top_k: int, top_p: float) -> torch.Tensor:
    """logits [n, B, l, V] fp32 -> idx [n, B, l]: the masking / softmax batched over members, one
    multinomial per member on its own generator (the call the reference makes per member)."""
    n, B, l, V = logits.shape
    probs = top_k_top_p_mask_(logits, top_k, top_p).softmax(dim=-1)
    return torch.stack([torch.multinomial(probs[k].view(-1, V), 1, replacement=True, generator=gens[k]).view(B, l)
                        for k in range(n)])


# ---------------------------------------------------------------------------------------
# population autoregressive inference
# ---------------------------------------------------------------------------------------


class VARPopulationInfer:
    """var.py:126-190 `autoregressive_infer_cfg` for n members at once (more_smooth=False)."""

    def __init__(self, var: VARTransformer, vae: VQVAEDecode):
        self.var, self.vae = var, vae
        self._kv: Dict[Tuple, List[torch.Tensor]] = {}

    def _caches(self, N2: int, dev) -> List[torch.Tensor]:
        a = self.var.arch
        key = (N2, str(dev))
        if key not in self._kv:
            self._kv = {key: [torch.empty((2, N2, a.heads, a.L, 64), dtype=torch.bfloat16, device=dev)
                              for _ in range(a.depth)]}
        return self._kv[key]

    @torch.no_grad()
    def run(self, label_B: torch.Tensor, n: int, g_seed: int, cfg: float, top_k: int, top_p: float,
            force_idx: Optional[List[torch.Tensor]] = None, keep_logits: bool = False):
        """label_B [B] long (shared by all members).  force_idx: optional per-scale [n*B, l] token maps
        that replace the sampled ones (teacher forcing, parity tests).  Returns (f_hat [n*B, Cvae, 16, 16]
        fp32, per-scale idx list, per-scale CFG logits list if keep_logits)."""
        var, a = self.var, self.var.arch
        C, H, hd, SN = a.C, a.heads, 64, len(a.patch_nums)
        dev = var.pos_1LC.device
        B = int(label_B.shape[0])
        B2, N2 = 2 * B, 2 * B * n
        gens = [torch.Generator(device=dev).manual_seed(int(g_seed)) for _ in range(n)]
        cond = var.class_emb(torch.cat((label_B, torch.full_like(label_B, a.num_classes)))).float()   # [2B, C]
        condN = F.silu(cond).to(torch.bfloat16).repeat(n, 1).contiguous()                             # [N2, C]
        adas = [blk.ada_lin[1](condN) for blk in var.blocks]                                         # [N2, 6C]
        ada_h = var.head_nm.ada_lin[1](condN)                                                         # [N2, 2C]
        lvl_pos = (var.lvl_embed(var.lvl_1L[0]) + var.pos_1LC[0]).float()                            # [L, C]
        first_l = a.patch_nums[0] ** 2
        x = (cond[:, None] + var.pos_start[0][None].float() + lvl_pos[None, :first_l])              # [2B, l0, C]
        x = x.to(torch.bfloat16).repeat(n, 1, 1).reshape(-1, C).contiguous()
        caches = self._caches(N2, dev)
        f_hat = torch.zeros((n * B, a.Cvae, a.patch_nums[-1], a.patch_nums[-1]), dtype=torch.float32, device=dev)
        code = self.vae.quantize.embedding.weight.float()
        idx_all, logits_all = [], []
        cur = 0
        for si, pn in enumerate(a.patch_nums):
            l = pn * pn
            ratio = si / (SN - 1)
            for blk, ada, kv in zip(var.blocks, adas, caches):
                at = blk.attn
                h = K.rownorm(x, a.norm_eps, layer=True, mscale=ada[:, 2 * C:3 * C], mshift=ada[:, 4 * C:5 * C],
                              rows_per_group=l)
                qkv = at.qkv(h).view(N2, l, 3, H, hd)
                q = F.normalize(qkv[:, :, 0].transpose(1, 2).float(), dim=-1).mul_(at.q_mul).to(torch.bfloat16)
                kv[0, :, :, cur:cur + l] = F.normalize(qkv[:, :, 1].transpose(1, 2).float(), dim=-1).to(torch.bfloat16)
                kv[1, :, :, cur:cur + l] = qkv[:, :, 2].transpose(1, 2)
                o = F.scaled_dot_product_attention(q, kv[0, :, :, :cur + l], kv[1, :, :, :cur + l], scale=1.0)
                o = o.transpose(1, 2).reshape(N2 * l, C).contiguous()
                K.gated_residual_(x, at.proj(o), ada[:, 0:C], rows_per_group=l)
                h = K.rownorm(x, a.norm_eps, layer=True, mscale=ada[:, 3 * C:4 * C], mshift=ada[:, 5 * C:6 * C],
                              rows_per_group=l)
                f = blk.ffn.fc2(F.gelu(blk.ffn.fc1(h), approximate="tanh"))
                K.gated_residual_(x, f, ada[:, C:2 * C], rows_per_group=l)
            cur += l
            h = K.rownorm(x, a.norm_eps, layer=True, mscale=ada_h[:, 0:C], mshift=ada_h[:, C:2 * C], rows_per_group=l)
            logits = var.head(h).float().view(n, 2, B, l, a.vocab_size)
            t = cfg * ratio
            logits = (1 + t) * logits[:, 0] - t * logits[:, 1]                                       # [n, B, l, V]
            if keep_logits:
                logits_all.append(logits.clone())
            if force_idx is not None:
                idx = force_idx[si].to(dev).view(n, B, l)
            else:
                idx = sample_population(logits, gens, top_k, top_p)
            idx_all.append(idx.reshape(n * B, l))
            h_BChw = code[idx.reshape(n * B, l)].transpose(1, 2).reshape(n * B, a.Cvae, pn, pn)
            f_hat, nxt = self.vae.next_autoregressive_input(si, SN, f_hat, h_BChw)
            if si != SN - 1:
                ln = a.patch_nums[si + 1] ** 2
                nxt = F.linear(nxt.reshape(n * B, a.Cvae, -1).transpose(1, 2), var.word_embed.weight.float(),
                               var.word_embed.bias.float()) + lvl_pos[cur:cur + ln]                 # [nB, l', C]
                x = nxt.view(n, 1, B, ln, C).expand(n, 2, B, ln, C).to(torch.bfloat16).reshape(-1, C).contiguous()
        return f_hat, idx_all, logits_all


# ---------------------------------------------------------------------------------------
# ES wrapper (models/VAR.py:27-334)
# ---------------------------------------------------------------------------------------


class VARClassGenerator:
    """models/VAR.py `VARClassGenerator`: `self.transformer` (= `self.var`) is the LoRA target;
    `generate(..., class_ids=...)` returns PIL images (or grouped lists) exactly as the reference;
    `generate_population(label_B, theta_pop, seed, cfg)` evaluates every member in one pass."""

    def __init__(self, model_depth: int = 16, device: str = "cuda:0", DTYPE: torch.dtype = torch.float16,
                 arch: Optional[VARArch] = None, num_classes: int = 1000, weight_seed: int = 0,
                 vae_chunk: int = 16):
        if arch is None:
            if model_depth not in {16, 20, 24, 30}:
                raise ValueError("model_depth must be one of {16, 20, 24, 30}")
            arch = VARArch(depth=model_depth, num_classes=num_classes)
        self.arch = arch
        self.device = str(device)
        self.DTYPE = DTYPE
        self.num_classes = arch.num_classes
        self.model_depth = arch.depth
        dev = torch.device(device)
        with torch.device(dev):
            self.var = VARTransformer(arch)
            self.vae = VQVAEDecode(arch)
        self.var.init_weights(weight_seed)
        self.vae.init_weights(weight_seed + 1)
        self._cast()
        self.transformer = self.var
        self.vae_chunk = vae_chunk
        self.ctx = PopulationContext()
        self.infer = VARPopulationInfer(self.var, self.vae)

    def _cast(self):
        """Frozen transformer linears bf16 (MFMA operands); VQVAE decoder bf16 channels-last."""
        for m in self.var.modules():
            if isinstance(m, LoRALinear):
                m.weight.data = m.weight.data.to(torch.bfloat16)
                if isinstance(m.bias, nn.Parameter):
                    m.bias.data = m.bias.data.to(torch.bfloat16)
        self.vae.decoder.to(torch.bfloat16).to(memory_format=torch.channels_last)
        self.var.refresh()

    def load_reference_state(self, var_state: Optional[dict] = None, vae_state: Optional[dict] = None):
        """Load the reference's checkpoints (var_d{depth}.pth, vae_ch160v4096z32.pth, already read with
        torch.load(weights_only=True)): keys as in the reference; the VQVAE encoder / quant_conv keys
        and training buffers are ignored; any missing decode-side key raises."""
        for mod, sd, skip in ((self.var, var_state, ("attn_bias_for_masking", "lvl_1L", "zero_k_bias")),
                              (self.vae, vae_state, ("encoder.", "quant_conv.", "ema_vocab_hit_SV"))):
            if sd is None:
                continue
            own = dict(mod.named_parameters())
            extra = [k for k in sd if k not in own and not any(s in k for s in skip)]
            missing = [k for k in own if k not in sd and ".lora_" not in k]
            if extra or missing:
                raise ValueError(f"state dict mismatch: missing {missing[:3]}, unexpected {extra[:3]}")
            with torch.no_grad():
                for k, p in own.items():
                    if k in sd:
                        if tuple(sd[k].shape) != tuple(p.shape):
                            raise ValueError(f"{k}: shape {tuple(sd[k].shape)} != {tuple(p.shape)}")
                        p.copy_(sd[k].to(p.device, p.dtype))
        self.var.refresh()
        for m in self.vae.modules():        # drop DConv2d's cached GEMM weight views
            if isinstance(m, DConv2d):
                m._wflat = None

    # ---- reference helpers -------------------------------------------------------------
    def _validate_labels(self, label: torch.Tensor) -> torch.Tensor:
        if label.ndim != 1:
            raise ValueError("class_ids must be 1D or 2D (flattened internally to 1D)")
        if (label < 0).any() or (label >= self.num_classes).any():
            raise ValueError(f"class_ids must be in [0, {self.num_classes - 1}]")
        return label

    def _flatten_class_ids(self, class_ids) -> Tuple[torch.Tensor, Optional[Tuple[int, int]]]:
        """models/VAR.py:206-242."""
        if isinstance(class_ids, torch.Tensor):
            if class_ids.ndim == 1:
                return self._validate_labels(class_ids.to(self.device, torch.long)), None
            if class_ids.ndim == 2:
                nb, bs = class_ids.shape
                return self._validate_labels(class_ids.reshape(-1).to(self.device, torch.long)), (int(nb), int(bs))
            raise ValueError("class_ids tensor must be 1D or 2D")
        if isinstance(class_ids, int):
            return self._validate_labels(torch.tensor([class_ids], device=self.device)), None
        if isinstance(class_ids, (list, tuple)) and len(class_ids) > 0 and isinstance(class_ids[0], (list, tuple)):
            batches = [list(map(int, b)) for b in class_ids]
            bs = len(batches[0])
            if bs == 0:
                raise ValueError("empty inner batch in class_ids")
            if any(len(b) != bs for b in batches):
                raise ValueError("All inner batches must have the same length")
            flat = torch.tensor([x for b in batches for x in b], device=self.device)
            return self._validate_labels(flat), (len(batches), bs)
        return self._validate_labels(torch.tensor([int(x) for x in class_ids], device=self.device)), None

    # ---- reference API -----------------------------------------------------------------
    @torch.no_grad()
    def generate(self, prompt_embeds=None, prompt_attention_mask=None, latents=None, seed: int = 0,
                 guidance_scale: float = 4.0, width_latent: int = 32, height_latent: int = 32, *, class_ids,
                 top_k: int = 900, top_p: float = 0.95, more_smooth: bool = False, return_grouped: bool = False,
                 output_type: str = "pil", **_):
        """models/VAR.py:264-334 for one member (the transformer's own LoRA parameters)."""
        if more_smooth:
            raise NotImplementedError("more_smooth (gumbel visualisation mode) is not on the ES path")
        label, shape = self._flatten_class_ids(class_ids)
        set_population(self.var, None)
        f_hat, _, _ = self.infer.run(label, 1, seed, guidance_scale, top_k, top_p)
        img = self.vae.fhat_to_img(f_hat, self.vae_chunk)
        if output_type == "pt":
            return img, None
        images = to_pil_var(img)
        if return_grouped:
            if shape is None:
                raise ValueError("return_grouped=True requires 2D class_ids input")
            nb, bs = shape
            return [images[i * bs:(i + 1) * bs] for i in range(nb)], None
        return images, None

    def encode_prompts(self, *a, **k):
        raise NotImplementedError("VARClassGenerator is class-conditional; no text prompt encoding.")

    # ---- engine API --------------------------------------------------------------------
    @torch.no_grad()
    def generate_population(self, label_B: torch.Tensor, theta_pop: torch.Tensor, seed: int, guidance_scale: float,
                            top_k: int = 900, top_p: float = 0.95) -> torch.Tensor:
        """All members of theta_pop [n, D]: images [n*B, 3, 256, 256] in [-1, 1], member-major."""
        n = theta_pop.shape[0]
        self.ctx.theta_pop, self.ctx.n_members = theta_pop, n
        set_population(self.var, self.ctx)
        try:
            f_hat, _, _ = self.infer.run(self._validate_labels(label_B), n, seed, guidance_scale, top_k, top_p)
        finally:
            set_population(self.var, None)
            self.ctx.theta_pop = None
        return self.vae.fhat_to_img(f_hat, self.vae_chunk)


def quantize_uint8_var(images: torch.Tensor) -> torch.Tensor:
    """models/VAR.py:190 + 245-259 on fp16 autocast output: recon.add_(1).mul_(0.5) in fp16, clamp to
    [0, 1], (x * 255.0) in fp16, .to(uint8) truncates.  Returns uint8-valued fp32 [n, 3, H, W]."""
    x = images.to(torch.float16)
    x = ((x + 1) * 0.5).clamp_(0, 1)
    return (x * 255.0).to(torch.uint8).float()


def to_pil_var(images: torch.Tensor) -> List:
    from PIL import Image
    arr = quantize_uint8_var(images).to(torch.uint8).permute(0, 2, 3, 1).cpu().numpy()
    return [Image.fromarray(a) for a in arr]
