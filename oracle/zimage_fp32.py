"""fp32 PyTorch restatement of ONE Z-Image-Turbo member generation (the reference's per-member path).

TEST INFRASTRUCTURE ONLY (imported by tests/ as the checker; the product never imports it).

The reference generates a member's images with diffusers' ZImagePipeline in bf16 (models/
zImageTurbo.py:96-101, 339-407) with the PEFT LoRA on to_q/to_k/to_v/linear/w1/w2/w3.  diffusers is
absent, so the architecture is the build's own restatement (hyperscalees_t2i_amd/zimage.py,
flux_vae.py, zimage_pipeline.py); this module runs that SAME architecture with the build's weights
upcast to fp32 in plain torch ops — PEFT formula per linear with member k's factors read from
theta_k, RMSNorm / tanh-gated sandwich norms, complex-rotation RoPE, exact softmax attention, the
flow-matching Euler steps, the VAE decoder with torch.group_norm — so the bf16 build's drift on every
stage can be measured (tests/test_gpu_zimage.py).  Parity with diffusers is UNPINNED.  It calls no
libeggroll kernel.
"""
from __future__ import annotations

import torch
import torch.nn.functional as F

from oracle.member_eval_fp32 import LoraLinear32, timestep_embedding

f32 = torch.float32


def _w(p):
    return None if p is None else p.detach().to(f32)


def rms(x, w, eps):
    return x * torch.rsqrt(x.pow(2).mean(-1, keepdim=True) + eps) * w


def rope(x, cos, sin):
    """x [B, S, H, D]; cos / sin [B, S, D/2]: (x0 + i x1)(cos + i sin) on adjacent pairs."""
    xc = torch.view_as_complex(x.reshape(*x.shape[:-1], -1, 2).contiguous())
    return torch.view_as_real(xc * torch.complex(cos, sin)[:, :, None, :]).flatten(-2)


def block(blk, x, cos, sin, key_bias, t_emb, theta_k, record):
    L = lambda m: LoraLinear32(m, theta_k)  # noqa: E731
    B, S, D = x.shape
    att = blk.attention
    if blk.modulation:
        m = F.linear(t_emb, _w(blk.adaLN_modulation[0].weight), _w(blk.adaLN_modulation[0].bias)).view(4, D)
        s_msa, g_msa, s_mlp, g_mlp = 1 + m[0], torch.tanh(m[1]), 1 + m[2], torch.tanh(m[3])
    else:
        s_msa = g_msa = s_mlp = g_mlp = 1.0
    n = rms(x, _w(blk.attention_norm1.weight), blk.attention_norm1.eps) * s_msa
    q = L(att.to_q)(n, record).view(B, S, att.heads, att.hd)
    k = L(att.to_k)(n, record).view(B, S, att.heads, att.hd)
    v = L(att.to_v)(n, record).view(B, S, att.heads, att.hd)
    q = rope(rms(q, _w(att.norm_q.weight), att.norm_q.eps), cos, sin)
    k = rope(rms(k, _w(att.norm_k.weight), att.norm_k.eps), cos, sin)
    o = F.scaled_dot_product_attention(q.transpose(1, 2), k.transpose(1, 2), v.transpose(1, 2), attn_mask=key_bias,
                                       scale=att.hd ** -0.5).transpose(1, 2).reshape(B, S, D)
    a = L(att.to_out[0])(o)
    x = x + g_msa * rms(a, _w(blk.attention_norm2.weight), blk.attention_norm2.eps)
    n = rms(x, _w(blk.ffn_norm1.weight), blk.ffn_norm1.eps) * s_mlp
    ff = blk.feed_forward
    h = F.silu(L(ff.w1)(n, record)) * L(ff.w3)(n, record)
    f = L(ff.w2)(h, record)
    return x + g_mlp * rms(f, _w(blk.ffn_norm2.weight), blk.ffn_norm2.eps)


def transformer_fp32(tr, lat, t, cap_feats, cap_lens, enc_index, theta_k, record=None):
    """One member: lat [b, C, H, W] fp32, t [1] model time, cap_feats [U, Lc, cap_dim], cap_lens [U],
    enc_index [b] -> velocity [b, C, H, W] fp32 (zimage.ZImageTransformer2DModel.forward in fp32)."""
    from hyperscalees_t2i_amd.zimage import rope_tables
    a = tr.config
    L = lambda m: LoraLinear32(m, theta_k)  # noqa: E731
    b, C, H, W = lat.shape
    U, Lc = cap_lens.numel(), cap_feats.shape[1]
    hp, wp = H // a.patch, W // a.patch
    N = hp * wp
    padl = (cap_lens + a.seq_multiple - 1) // a.seq_multiple * a.seq_multiple   # each caption's padded length
    te = tr.t_embedder
    t_emb = F.linear(F.silu(F.linear(timestep_embedding(t * a.t_scale), _w(te.mlp[0].weight), _w(te.mlp[0].bias))),
                     _w(te.mlp[2].weight), _w(te.mlp[2].bias))
    x = L(tr.all_x_embedder[f"{a.patch}-1"])(tr.patchify(lat.to(f32)))
    ce = tr.cap_embedder
    cap = L(ce[1])(rms(cap_feats.to(f32), _w(ce[0].weight), ce[0].eps))
    tok = torch.arange(Lc, device=lat.device)[None, :]
    cap = torch.where((tok < cap_lens[:, None])[..., None], cap, _w(tr.cap_pad_token).view(1, 1, -1))
    img_pos, cap_pos = tr.positions(padl, Lc, hp, wp)
    ci, si = rope_tables(a, img_pos[enc_index])
    cc, sc = rope_tables(a, cap_pos.expand(U, Lc, 3))
    # one batch with a key mask past each caption's padded length (the build groups images instead)
    cap_bias = torch.zeros(U, Lc, device=lat.device).masked_fill(tok >= padl[:, None], float("-inf"))
    for blk in tr.noise_refiner:
        x = block(blk, x, ci, si, None, t_emb, theta_k, record)
    for blk in tr.context_refiner:
        cap = block(blk, cap, cc, sc, cap_bias[:, None, None, :], None, theta_k, record)
    u = torch.cat((x, cap[enc_index]), 1)
    ub = torch.cat((torch.zeros(b, N, device=lat.device), cap_bias[enc_index]), 1)[:, None, None, :]
    cu, su = torch.cat((ci, cc[enc_index]), 1), torch.cat((si, sc[enc_index]), 1)
    for blk in tr.layers:
        u = block(blk, u, cu, su, ub, t_emb, theta_k, record)
    fl = tr.all_final_layer[f"{a.patch}-1"]
    scale = F.linear(F.silu(t_emb), _w(fl.adaLN_modulation[1].weight), _w(fl.adaLN_modulation[1].bias))
    xo = u[:, :N]
    n = (xo - xo.mean(-1, keepdim=True)) * torch.rsqrt(xo.var(-1, unbiased=False, keepdim=True) + 1e-6) * (1 + scale)
    out = L(fl.linear)(n, record)
    return tr.unpatchify(out, H, W)


def vae_fp32(vae, z, theta_k=None):
    """flux_vae.FluxVAEDecoder in fp32 (NCHW, torch.group_norm); theta_k: member k's theta when the decoder
    carries the VAE LoRA (mid-block to_q / to_k / to_v / to_out.0, PEFT formula)."""
    def conv(m, x):
        return F.conv2d(x, _w(m.weight), _w(m.bias), padding=m.ks // 2)

    def gn(m, x, silu=True):
        y = F.group_norm(x, m.groups, _w(m.weight), _w(m.bias), m.eps)
        return F.silu(y) if silu else y

    def res(r, x):
        h = conv(r.conv2, gn(r.norm2, conv(r.conv1, gn(r.norm1, x))))
        return h + (x if r.conv_shortcut is None else conv(r.conv_shortcut, x))

    def attn(m, x):
        B, C, H, W = x.shape
        n = gn(m.group_norm, x, silu=False).flatten(2).transpose(1, 2)                  # [B, HW, C]
        q, k, v = (LoraLinear32(mm, theta_k)(n)[:, None] for mm in (m.to_q, m.to_k, m.to_v))
        o = F.scaled_dot_product_attention(q, k, v, scale=C ** -0.5)[:, 0]
        return LoraLinear32(m.to_out[0], theta_k)(o).transpose(1, 2).reshape(B, C, H, W) + x

    x = conv(vae.conv_in, z.to(f32))
    x = attn(vae.mid[1], res(vae.mid[0], x))
    x = res(vae.mid[2], x)
    for blk in vae.up_blocks:
        for r in blk.resnets:
            x = res(r, x)
        if blk.upsample is not None:
            x = conv(blk.upsample, F.interpolate(x, scale_factor=2, mode="nearest"))
    return conv(vae.conv_out, gn(vae.conv_norm_out, x))


def generate_fp32(model, theta_k, embeds, prompt_index, seed, width_px, height_px, steps, record=None,
                  vae_lora: bool = False):
    """One member's images: the build's ZImageTurboES inputs (distinct prompt embeddings, image ->
    prompt index, per-image seeded latents, flow_sigmas) through the fp32 transformer and VAE."""
    from hyperscalees_t2i_amd.zimage_pipeline import flow_sigmas
    cap, lens = model._captions(embeds)
    x = model._latents(prompt_index.numel(), seed, height_px, width_px)
    sig = flow_sigmas(steps)
    vel = []
    for i in range(steps):
        t = torch.full((1,), 1.0 - sig[i], device=x.device, dtype=f32)
        v = transformer_fp32(model.transformer, x, t, cap.to(f32), lens, prompt_index, theta_k,
                             record if i == 0 else None)
        vel.append(v)
        x = x + (sig[i + 1] - sig[i]) * (-v)
    z = x / model.vae.scaling_factor + model.vae.shift_factor
    return vel, vae_fp32(model.vae, z, theta_k if vae_lora else None)
