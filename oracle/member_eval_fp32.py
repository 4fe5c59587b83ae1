"""fp32 PyTorch restatement of ONE member evaluation (the reference's per-member path).

TEST INFRASTRUCTURE ONLY (imported by tests/ as the checker; the product never imports it).

The reference evaluates a member as `theta_k -> unflatten_to_params -> generate_flat ->
compute_all_rewards` in fp32 (transformer and VAE loaded in fp32, models/SanaSprint.py:34-49;
CLIP / PickScore models in their checkpoint dtype, rewards.py:32-60), one member at a time
(unifed_es.py:159-215).  The build runs the same member-eval in bf16 on hand-written kernels with
all members batched.  This module restates the member-eval with the build's OWN weights (the bf16
parameters upcast exactly to fp32) in plain fp32 torch ops — PEFT LoRA formula per linear
(y = x W^T + b + s (x A_k^T) B_k^T, es_backend.py:193-200), the same architecture as
hyperscalees_t2i_amd/sana.py + dcae.py + rewards.py, the one-step SCM math with the reference's
fp16 casts (models/SanaSprint.py:83-153) — so the bf16 drift of every tensor on the path (LoRA
activations, transformer output, image, rewards, S, ranks) can be measured and bounded
(tests/test_gpu_parity_fp32.py).  It calls no libeggroll kernel.
"""
from __future__ import annotations

import copy
import math
from typing import Dict, List, Optional

import torch
import torch.nn.functional as F

f32 = torch.float32


def _w(p):
    return None if p is None else p.detach().to(f32)


# ---------------------------------------------------------------------------------------------
# primitives (the build's fused kernels, restated in fp32)
# ---------------------------------------------------------------------------------------------


def rownorm(x, eps, layer=False, w=None, b=None, mscale=None, mshift=None, act=None, res=None):
    """eggroll_rownorm: (x - mean*layer) * rsqrt(var + eps) [*w] [*(1+mscale)] [+mshift] [+b] [act] [+res]."""
    mean = x.mean(-1, keepdim=True) if layer else 0.0
    xc = x - mean
    y = xc * torch.rsqrt(xc.pow(2).mean(-1, keepdim=True) + eps)
    if w is not None:
        y = y * w
    if mscale is not None:
        y = y * (1.0 + mscale)
    if mshift is not None:
        y = y + mshift
    if b is not None:
        y = y + b
    if act == "relu":
        y = F.relu(y)
    elif act == "silu":
        y = F.silu(y)
    if res is not None:
        y = y + res
    return y


def linear_attention(q, k, v, relu_qk: bool):
    """ReLU linear attention, head dim 32: q/k/v [B, N, heads, 32] -> [B, N, heads*32]."""
    if relu_qk:
        q, k = F.relu(q), F.relu(k)
    kv = torch.einsum("bnhi,bnhj->bhij", v, k)
    ks = k.sum(1)                                              # [B, h, 32]
    num = torch.einsum("bnhj,bhij->bnhi", q, kv)
    den = torch.einsum("bnhj,bhj->bnh", q, ks)[..., None] + 1e-15
    o = num / den
    return o.reshape(q.shape[0], q.shape[1], -1)


def dwconv_nhwc(x, w_t, bias, ks, pre_silu, glu):
    """eggroll_dwconv_nhwc: x [B,H,W,C], w_t [ks*ks, C] tap-major."""
    C = x.shape[-1]
    if pre_silu:
        x = F.silu(x)
    w = w_t.t().reshape(C, 1, ks, ks)
    y = F.conv2d(x.permute(0, 3, 1, 2), w, bias, padding=ks // 2, groups=C).permute(0, 2, 3, 1)
    if glu:
        h = C // 2
        y = y[..., :h] * F.silu(y[..., h:])
    return y


def conv3x3(x, w, b):  # NHWC
    return F.conv2d(x.permute(0, 3, 1, 2), w, b, padding=1).permute(0, 2, 3, 1)


# ---------------------------------------------------------------------------------------------
# transformer (hyperscalees_t2i_amd/sana.py architecture)
# ---------------------------------------------------------------------------------------------


class LoraLinear32:
    """PEFT lora.Linear forward in fp32 with member k's (A_k, B_k) read from theta_k."""

    def __init__(self, m, theta_k: Optional[torch.Tensor]):
        self.W, self.b = _w(m.weight), _w(m.bias)
        self.A = self.B = None
        if m.r and theta_k is not None:
            self.A = theta_k[m.theta_off_A:m.theta_off_A + m.r * m.in_features].view(m.r, m.in_features)
            self.B = theta_k[m.theta_off_B:m.theta_off_B + m.out_features * m.r].view(m.out_features, m.r)
            self.s = m.scale

    def __call__(self, x, record: Optional[list] = None):
        y = F.linear(x, self.W, self.b)
        if self.A is not None:
            t = F.linear(x, self.A)
            y = y + F.linear(t, self.B) * self.s
        if record is not None:
            record.append(y)
        return y


def timestep_embedding(t, dim=256, max_period=10000.0):
    half = dim // 2
    exponent = -math.log(max_period) * torch.arange(half, dtype=f32, device=t.device) / half
    emb = t.to(f32)[:, None] * torch.exp(exponent)[None, :]
    return torch.cat([torch.cos(emb), torch.sin(emb)], dim=-1)


def transformer_fp32(tr, theta_k, hidden_states, timestep, enc_states, enc_mask, guidance,
                     record: Optional[list] = None, rnd=()):
    """SanaTransformer2DModel.forward of the build, fp32, member k's LoRA.
    rnd (drift attribution, tools/drift_probe.py): classes of points rounded to bf16 as the build
    stores them — "x" the residual stream after every update, "lin_in" every GEMM operand built from
    activations, "lin_out" every linear's output, "norm" row-norm outputs, "attn" attention outputs,
    "out" the transformer output, "mods" the AdaLN modulation (scale_shift_table + timestep6, a bf16 add
    in the build), "temb" the time / guidance embedding chain.  Empty: pure fp32."""
    bf = lambda t, c: t.to(torch.bfloat16).to(f32) if c in rnd else t  # noqa: E731

    class _L(LoraLinear32):
        def __call__(self, x, record=None):
            return bf(super().__call__(bf(x, "lin_in"), record), "lin_out")
    L = lambda m: (_L if rnd else LoraLinear32)(m, theta_k)  # noqa: E731
    a = tr.config
    B, C, H, W = hidden_states.shape
    x = hidden_states.to(f32).permute(0, 2, 3, 1).reshape(B, H * W, C)
    x = bf(F.linear(x, _w(tr.patch_w), _w(tr.patch_b)), "x")
    te = tr.time_embed
    te_ = lambda t: bf(t, "temb")  # noqa: E731
    t = te_(L(te.timestep_embedder.linear_2)(te_(F.silu(L(te.timestep_embedder.linear_1)(
        te_(timestep_embedding(timestep)), record))), record))
    g = te_(L(te.guidance_embedder.linear_2)(te_(F.silu(L(te.guidance_embedder.linear_1)(
        te_(timestep_embedding(guidance)), record))), record))
    cond = te_(t + g)
    timestep6 = L(te.linear)(te_(F.silu(cond)), record)
    cp = tr.caption_projection
    enc = L(cp.linear_2)(F.gelu(L(cp.linear_1)(enc_states.to(f32), record), approximate="tanh"), record)
    enc = bf(rownorm(enc, tr.caption_norm.eps, w=_w(tr.caption_norm.weight)), "norm")
    mask_bias = ((1.0 - enc_mask.to(f32)) * -10000.0).view(B, 1, 1, -1)
    N = H * W
    for blk in tr.transformer_blocks:
        mods = bf(_w(blk.scale_shift_table)[None] + timestep6.view(B, 6, -1), "mods")
        n = bf(rownorm(x, blk.eps, layer=True, mscale=mods[:, 1:2], mshift=mods[:, 0:1]), "norm")
        at = blk.attn1
        q = bf(rownorm(L(at.to_q)(n, record), at.norm_q.eps, w=_w(at.norm_q.weight), act="relu"), "norm")
        k = bf(rownorm(L(at.to_k)(n, record), at.norm_k.eps, w=_w(at.norm_k.weight), act="relu"), "norm")
        v = L(at.to_v)(n, record)
        sh = (B, N, at.heads, at.head_dim)
        o = bf(linear_attention(q.view(sh), k.view(sh), v.view(sh), relu_qk=False), "attn")
        x = bf(x + mods[:, 2:3] * L(at.to_out[0])(o, record), "x")
        ca = blk.attn2
        Lc = enc.shape[1]
        q = bf(rownorm(L(ca.to_q)(x, record), ca.norm_q.eps, w=_w(ca.norm_q.weight)), "norm").view(B, N, ca.heads,
                                                                                                    ca.head_dim)
        k = bf(rownorm(L(ca.to_k)(enc, record), ca.norm_k.eps, w=_w(ca.norm_k.weight)), "norm").view(B, Lc, ca.heads,
                                                                                                      ca.head_dim)
        v = L(ca.to_v)(enc, record).view(B, Lc, ca.heads, ca.head_dim)
        s = torch.einsum("bnhd,blhd->bhnl", q, k) * ca.head_dim ** -0.5 + mask_bias
        o = bf(torch.einsum("bhnl,blhd->bnhd", torch.softmax(s, -1), v).reshape(B, N, -1), "attn")
        x = bf(x + L(ca.to_out[0])(o, record), "x")
        n = bf(rownorm(x, blk.eps, layer=True, mscale=mods[:, 4:5], mshift=mods[:, 3:4]), "norm")
        ff = blk.ff
        h = bf(F.linear(n, _w(ff.w_inv), _w(ff.b_inv)), "lin_out").view(B, H, W, -1)
        gl = bf(dwconv_nhwc(h, _w(ff.w_dw), _w(ff.b_dw), 3, pre_silu=True, glu=True), "attn")
        x = bf(x + mods[:, 5:6] * bf(F.linear(gl.reshape(B, N, -1), _w(ff.w_point)), "lin_out"), "x")
    mods = bf(_w(tr.scale_shift_table)[None] + cond[:, None], "mods")
    x = bf(rownorm(x, a.norm_eps, layer=True, mscale=mods[:, 1:2], mshift=mods[:, 0:1]), "norm")
    x = bf(L(tr.proj_out)(x, record), "out")
    return x.view(B, H, W, a.out_channels).permute(0, 3, 1, 2)


# ---------------------------------------------------------------------------------------------
# DC-AE decoder (hyperscalees_t2i_amd/dcae.py architecture; literal nearest-upsample up-blocks)
# ---------------------------------------------------------------------------------------------


def _upshortcut(x, cout):
    """pixel_shuffle(repeat_interleave(x, 4*cout/cin, channel), 2), NHWC."""
    B, H, W, Cin = x.shape
    rep = x.repeat_interleave(4 * cout // Cin, dim=-1)                     # [B,H,W,4*cout]
    y = F.pixel_shuffle(rep.permute(0, 3, 1, 2), 2)                        # [B,cout,2H,2W]
    return y.permute(0, 2, 3, 1)


def dcae_fp32(vae, z, rnd=()):
    """rnd (drift attribution): "dx" rounds the residual stream after every block ("dx_vit" / "dx_res" /
    "dx_up": only after the EfficientViT blocks + conv_in / the ResBlocks / the up-blocks), "dact" every
    other activation the build stores in bf16 (conv / GEMM outputs, attention outputs, the input)."""
    from hyperscalees_t2i_amd.dcae import EfficientViTBlock, ResBlock, UpBlock
    _bf = lambda t, c: t.to(torch.bfloat16).to(f32) if c in rnd else t  # noqa: E731
    kind = {"vit": "dx_vit", "res": "dx_res", "up": "dx_up"}

    def bf(t, c, k=None):
        if c == "dx" and k is not None and kind[k] in rnd:
            return t.to(torch.bfloat16).to(f32)
        return _bf(t, c)
    zt = bf(z.to(f32).permute(0, 2, 3, 1), "dact")
    x = bf(conv3x3(zt, _w(vae.conv_in.weight), _w(vae.conv_in.bias)) + zt.repeat_interleave(vae.in_repeats, dim=-1), "dx",
           "vit")
    for st in vae.stages:
        for blk in st:
            if isinstance(blk, UpBlock):
                cout = blk.conv.weight.shape[0]
                up = F.interpolate(x.permute(0, 3, 1, 2), scale_factor=2, mode="nearest").permute(0, 2, 3, 1)
                x = bf(conv3x3(up, _w(blk.conv.weight), _w(blk.conv.bias)) + _upshortcut(x, cout), "dx", "up")
            elif isinstance(blk, ResBlock):
                h = bf(F.silu(conv3x3(x, _w(blk.conv1.weight), _w(blk.conv1.bias))), "dact")
                h = conv3x3(h, _w(blk.conv2.weight), None)
                x = bf(rownorm(h, blk.norm.eps, w=_w(blk.norm.weight), b=_w(blk.norm.bias), res=x), "dx", "res")
            elif isinstance(blk, EfficientViTBlock):
                x = bf(_msla(blk.attn, x, bf), "dx", "vit")
                c = blk.conv_out
                h = bf(F.linear(x, _w(c.w_inv), _w(c.b_inv)), "dact")
                g = bf(dwconv_nhwc(h, _w(c.w_dw), _w(c.b_dw), 3, pre_silu=True, glu=True), "dact")
                x = bf(rownorm(bf(F.linear(g, _w(c.w_point)), "dact"), c.norm.eps, w=_w(c.norm.weight),
                               b=_w(c.norm.bias), res=x), "dx", "vit")
            else:
                raise TypeError(type(blk))
    x = bf(rownorm(x, vae.norm_out.eps, w=_w(vae.norm_out.weight), b=_w(vae.norm_out.bias), act="relu"), "dact")
    return conv3x3(x, _w(vae.conv_out.weight), _w(vae.conv_out.bias)).permute(0, 3, 1, 2)


def _msla(at, x, bf=lambda t, c: t):
    B, H, W, C = x.shape
    hd, heads = at.hd, at.heads
    qkv = bf(F.linear(x, _w(at.w_qkv)), "dact")                           # [B,H,W,3*inner], head h: [q|k|v]
    outs = []
    t = qkv.reshape(B, H * W, heads, 3, hd)
    outs.append(bf(linear_attention(t[:, :, :, 0], t[:, :, :, 1], t[:, :, :, 2], relu_qk=True), "dact"))
    for ks, wdw, wpw in zip(at.scales, at.ms_dw, at.ms_pw):
        d = dwconv_nhwc(qkv, _w(wdw), None, ks, pre_silu=False, glu=False)
        g = d.reshape(B * H * W, 3 * heads, hd)
        pg = bf(torch.einsum("ngi,goi->ngo", g, _w(wpw)), "dact").reshape(B, H * W, heads, 3, hd)
        outs.append(bf(linear_attention(pg[:, :, :, 0], pg[:, :, :, 1], pg[:, :, :, 2], relu_qk=True), "dact"))
    y = bf(F.linear(torch.cat(outs, -1).view(B, H, W, -1), _w(at.w_out)), "dact")
    n = at.norm_out
    return rownorm(y, n.eps, w=_w(n.weight), b=_w(n.bias), res=x)


# ---------------------------------------------------------------------------------------------
# one-step generation + rewards
# ---------------------------------------------------------------------------------------------


def generate_fp32(es_model, theta_k, prompt_embeds, prompt_mask, latents, guidance_scale: float,
                  record: Optional[list] = None, rnd=(), drnd=(), decode_chunk: Optional[int] = None):
    """models/SanaSprint.py:96-160 with the build's weights in fp32: (eps_pred, image); rnd: see
    transformer_fp32; decode_chunk: decode that many images at a time (the decoder is per image, so
    chunking changes no value; it bounds the fp32 feature maps at 1024 px)."""
    b = latents.shape[0]
    sd = es_model.sigma_data
    lmi = latents / sd
    t = torch.tensor(1.571, device=latents.device, dtype=f32).expand(b)
    scm = torch.sin(t) / (torch.cos(t) + torch.sin(t))
    se = scm.view(-1, 1, 1, 1)
    guidance = torch.full((b,), guidance_scale, device=latents.device, dtype=es_model.DTYPE)
    guidance = guidance * es_model.transformer_config.guidance_embeds_scale
    eps = transformer_fp32(es_model.transformer, theta_k, lmi.to(f32), scm, prompt_embeds.to(f32), prompt_mask,
                           guidance.to(f32), record, rnd)
    return eps, decode_fp32(es_model, eps, latents, drnd, decode_chunk)


def decode_fp32(es_model, eps, latents, drnd=(), chunk: Optional[int] = None):
    """models/SanaSprint.py:133-160 after the transformer: nan_to_num, SCM combine (the reference's fp16
    casts), x0, fp32 DC-AE decode.  Also used on the build's bf16 transformer output to split the image
    drift into its transformer and DC-AE parts."""
    if chunk is not None and eps.shape[0] > chunk:
        return torch.cat([decode_fp32(es_model, eps[i:i + chunk], latents[i:i + chunk], drnd)
                          for i in range(0, eps.shape[0], chunk)])
    sd = es_model.sigma_data
    lmi = latents / sd
    se = (torch.sin(torch.tensor(1.571, device=latents.device, dtype=f32))
          / (torch.cos(torch.tensor(1.571, device=latents.device, dtype=f32))
             + torch.sin(torch.tensor(1.571, device=latents.device, dtype=f32)))).view(1, 1, 1, 1)
    eps = torch.nan_to_num(eps.to(f32), nan=0.0, posinf=0.0, neginf=0.0)
    pred = ((1 - 2 * se) * lmi + (1 - 2 * se + 2 * se ** 2) * eps.to(lmi.dtype)) / torch.sqrt(se ** 2 + (1 - se) ** 2)
    pred = pred.float() * sd
    x0 = (0.267 * latents - 0.964 * pred) / sd
    return dcae_fp32(es_model.vae, x0.to(f32) / es_model.vae.scaling_factor, drnd)


class Rewards32:
    """RewardModels with fp32 copies of the same CLIP / PickScore weights."""

    def __init__(self, rewards):
        self.clip = copy.deepcopy(rewards.clip).float()
        self.pick = copy.deepcopy(rewards.pick).float()
        self.mix_weights = rewards.mix_weights
        self.tokenize = rewards.tokenize    # the same token ids as the build (synthetic or the local BPE)

    @torch.no_grad()
    def prompt_features(self, prompts: List[str]) -> Dict[str, torch.Tensor]:
        dev = next(self.clip.parameters()).device
        ids_c, mask_c, ids_p, mask_p = (t.to(dev) for t in self.tokenize(prompts))
        tc = self.clip.text_projection(self.clip.text_model(input_ids=ids_c, attention_mask=mask_c).pooler_output)
        tc = tc / tc.norm(dim=-1, keepdim=True).clamp_min(1e-6)
        tp = self.pick.text_projection(self.pick.text_model(input_ids=ids_p, attention_mask=mask_p).pooler_output)
        tp = tp / tp.norm(dim=-1, keepdim=True)
        return {"clip_aes": tc[0], "clip_neg": tc[1], "clip_prompt": tc[2:], "pick_prompt": tp}

    @torch.no_grad()
    def score(self, images, prompt_index, feats) -> Dict[str, torch.Tensor]:
        from hyperscalees_t2i_amd.rewards import clip_preprocess, postprocess_uint8, split_mix_weights
        px = clip_preprocess(postprocess_uint8(images))
        ic = self.clip.visual_projection(self.clip.vision_model(pixel_values=px).pooler_output)
        ic = ic / ic.norm(dim=-1, keepdim=True).clamp_min(1e-6)
        ip = self.pick.visual_projection(self.pick.vision_model(pixel_values=px).pooler_output)
        ip = ip / ip.norm(dim=-1, keepdim=True)
        aes = (ic @ feats["clip_aes"] + 1.0) / 2.0
        txt = ((ic * feats["clip_prompt"][prompt_index]).sum(-1) + 1.0) / 2.0
        noart = 1.0 - (ic @ feats["clip_neg"] + 1.0) / 2.0
        pick = self.pick.logit_scale.exp() * (ip * feats["pick_prompt"][prompt_index]).sum(-1)
        w_aes, w_txt, w_no, w_pick = split_mix_weights(self.mix_weights)
        comb = w_aes * aes + w_txt * txt + w_no * noart + w_pick * pick
        return {"clip_aesthetic": aes, "clip_text": txt, "no_artifacts": noart, "pickscore": pick, "combined": comb}
