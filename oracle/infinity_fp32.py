"""fp32 PyTorch restatement of ONE Infinity member's autoregressive pass (the reference's per-member path).

TEST INFRASTRUCTURE ONLY (imported by tests/ as the checker; the product never imports it).

The reference samples a member's images with the Infinity repo's `autoregressive_infer_cfg` under bf16
autocast (models/Infinity.py:509-537) with PEFT LoRA on fc1.  The Infinity repo is not vendored, so the
architecture is the build's own restatement (hyperscalees_t2i_amd/infinity.py); this module runs that
SAME architecture on the build's weights upcast to fp32 in plain torch ops — per-member PEFT formula on
fc1 from theta_k, LayerNorm / AdaLN with the shared table, cosine self-attention with exact L2
normalisation and complex-rotation 2-D RoPE over the cached scales, cross-attention to each image's own
text (no padding), per-scale CFG — and returns the per-scale CFG logits given forced bits (teacher
forcing), so the bf16 population build's drift can be measured per scale (tests/test_gpu_infinity.py).
Parity with the Infinity repo is UNPINNED.  It calls no libeggroll kernel.
"""
from __future__ import annotations

import math

import torch
import torch.nn.functional as F

from oracle.member_eval_fp32 import LoraLinear32

f32 = torch.float32


def _w(p):
    return None if p is None else p.detach().to(f32)


def ln(x, eps, w=None, b=None):
    return F.layer_norm(x, x.shape[-1:], _w(w), _w(b), eps)


def rope(x, cos, sin):
    """x [S, H, D]; cos / sin [S, D/2]: (x0 + i x1)(cos + i sin) on adjacent pairs."""
    xc = torch.view_as_complex(x.reshape(*x.shape[:-1], -1, 2).contiguous())
    return torch.view_as_real(xc * torch.complex(cos, sin)[:, None, :]).flatten(-2)


def member_logits_fp32(tr, kv_list, lens, prompt_index, theta_k, schedule, cfg_list, tau_list, force_bits):
    """One member: distinct prompts kv_list [L_u, Ct5] / lens, prompt_index [B], theta_k [D] fp32,
    force_bits per scale [B, l, d_tok] -> per-scale CFG logits [B, l*d_tok, 2] fp32."""
    from hyperscalees_t2i_amd.infinity import bits_to_codes, codes_to_tokens, rope2d_tables
    a = tr.arch
    C, H, hd = a.C, a.num_heads, a.head_dim
    dev = tr.pos_start.device
    L = lambda m: LoraLinear32(m, theta_k)  # noqa: E731
    B = int(prompt_index.numel())
    # per-row text (cond rows 0..B-1, uncond rows B..2B-1), exact lengths
    texts = []
    for half in (0, 1):
        for j in range(B):
            u = int(prompt_index[j])
            Lu = int(lens[u])
            t = kv_list[u][:Lu].to(dev, f32) if half == 0 else _w(tr.cfg_uncond[:Lu])
            texts.append(t * torch.rsqrt(t.pow(2).mean(-1, keepdim=True) + tr.text_norm.eps) * _w(tr.text_norm.weight))
    pool = tr.text_proj_for_sos
    Hp = pool.heads
    sos, ca_tok = [], []
    for t in texts:
        kv = L(pool.mat_kv)(t).view(-1, 2, Hp, C // Hp)
        q = _w(pool.query).view(Hp, 1, C // Hp)
        att = torch.softmax(q @ kv[:, 0].permute(1, 2, 0) / math.sqrt(C // Hp), -1)         # [Hp, 1, Lu]
        sos.append(L(pool.proj)((att @ kv[:, 1].transpose(0, 1)).reshape(C)))
        ca = tr.text_proj_for_ca
        ca_tok.append(L(ca[2])(F.gelu(L(ca[0])(t), approximate="tanh")))
    sos = torch.stack(sos)                                                                    # [2B, C]
    shared = L(tr.shared_ada_lin[1])(F.silu(sos)).view(2 * B, 6, C)
    ada_h = L(tr.head_nm.ada_lin[1])(F.silu(sos))
    blocks = tr.blocks()
    per_chunk = len(blocks) // len(tr.block_chunks)
    side = schedule[-1][1]
    vside = side * (2 if a.spatial_patchify else 1)
    x = sos + _w(tr.pos_start).view(1, C)
    x = x[:, None, :]                                                                         # [2B, 1, C]
    cache = [([], []) for _ in blocks]
    summed = torch.zeros((B, a.codebook_dim, vside, vside), dtype=f32, device=dev)
    out = []
    for si, (_, h, w) in enumerate(schedule):
        l = h * w
        cos, sin = rope2d_tables(a, h, w, side, dev)
        for bi, blk in enumerate(blocks):
            if bi % per_chunk == 0:
                x = x + _w(tr.lvl_embed[si]).view(1, 1, C)
            g1, g2, s1, s2, h1, h2 = (_w(blk.ada_gss).view(1, 6, C) + shared).unbind(1)
            n = ln(x, a.norm_eps) * (1 + s1[:, None]) + h1[:, None]
            qkv = L(blk.sa.mat_qkv)(n).view(2 * B, l, 3, H, hd)
            sm = _w(blk.sa.scale_mul_1H11).view(H).clamp(max=math.log(100.0)).exp()
            att_out = []
            for r in range(2 * B):
                q = rope(F.normalize(qkv[r, :, 0], dim=-1), cos, sin)
                k = rope(F.normalize(qkv[r, :, 1], dim=-1), cos, sin)
                if len(cache[bi][0]) <= r:
                    cache[bi][0].append(k)
                    cache[bi][1].append(qkv[r, :, 2])
                else:
                    cache[bi][0][r] = torch.cat((cache[bi][0][r], k))
                    cache[bi][1][r] = torch.cat((cache[bi][1][r], qkv[r, :, 2]))
                ks, vs = cache[bi][0][r], cache[bi][1][r]
                logit = torch.einsum("qhd,khd->hqk", q, ks) * sm.view(H, 1, 1)
                att_out.append(torch.einsum("hqk,khd->qhd", torch.softmax(logit, -1), vs).reshape(l, C))
            x = x + g1[:, None] * L(blk.sa.proj)(torch.stack(att_out))
            n = ln(x, a.norm_eps, blk.ca_norm.weight, blk.ca_norm.bias)
            q = L(blk.ca.mat_q)(n).view(2 * B, l, H, hd)
            ca_out = []
            for r in range(2 * B):
                kv = L(blk.ca.mat_kv)(ca_tok[r]).view(-1, 2, H, hd)
                logit = torch.einsum("qhd,khd->hqk", q[r], kv[:, 0]) / math.sqrt(hd)
                ca_out.append(torch.einsum("hqk,khd->qhd", torch.softmax(logit, -1), kv[:, 1]).reshape(l, C))
            x = x + L(blk.ca.proj)(torch.stack(ca_out))
            n = ln(x, a.norm_eps) * (1 + s2[:, None]) + h2[:, None]
            x = x + g2[:, None] * L(blk.ffn.fc2)(F.gelu(L(blk.ffn.fc1)(n), approximate="tanh"))
        hn = ln(x, a.norm_eps) * (1 + ada_h[:, None, :C]) + ada_h[:, None, C:]
        lg = L(tr.head)(hn).view(2, B, l * a.d_tok, 2) / float(tau_list[si])
        cfg = float(cfg_list[si])
        out.append(cfg * lg[0] + (1.0 - cfg) * lg[1])
        codes = bits_to_codes(force_bits[si].to(dev).view(B, l, a.d_tok), a, h, w)
        if si != len(schedule) - 1:
            summed = summed + F.interpolate(codes, size=(vside, vside), mode="bilinear", align_corners=False)
            _, h2_, w2_ = schedule[si + 1]
            vh = h2_ * (2 if a.spatial_patchify else 1)
            e = L(tr.word_embed)(codes_to_tokens(F.interpolate(summed, size=(vh, vh), mode="area"), a))
            x = torch.cat((e, e))
    return out
