"""CLIP vision tower for the batched reward path (rewards.py:66-158 of the reference runs
transformers' CLIPModel.get_image_features once per image).

Same weights and the same arithmetic as transformers' CLIPVisionModel + visual_projection
(patch conv -> [CLS] + positions -> pre-LN -> pre-norm encoder layers -> post-LN of [CLS] ->
projection), restated for throughput on every image of every local member at once:
  * q / k / v projections fused into one GEMM per layer ([3C, C] weight, concatenated biases);
  * the patch-embedding conv (stride = kernel) as a patch reshape + GEMM;
  * the LAST layer runs its attention output, MLP and residuals on the [CLS] rows only — the only
    rows get_image_features reads (its keys / values still come from every token);
  * one batch for all images (no per-image or per-chunk model calls).
Precision (`fp32_residual`, default on): GEMM operands are bf16 (MFMA) with fp32 accumulation,
but everything that carries the signal from layer to layer is fp32 — the patch embedding, the
residual stream h, every LayerNorm (fp32 in, bf16 out for the next GEMM), each block's output added
to h in fp32, the post-LN and the projection.  The reference runs these towers in fp32
(rewards.py:32-60, from_pretrained defaults); a bf16 residual stream rounds h 64 times per CLIP-H
image and was the largest single term of the member-eval S drift.  fp32_residual=False
is the plain bf16 module (kept for A/B).
"""
from __future__ import annotations

from typing import List

import torch
import torch.nn.functional as F

ACT = {"gelu": lambda x: F.gelu(x), "quick_gelu": lambda x: x * torch.sigmoid(1.702 * x),
       "gelu_new": lambda x: F.gelu(x, approximate="tanh")}


class CLIPVisionTower:
    def __init__(self, model, pad_head_dim: bool = False, use_kernel: bool = True, fp32_residual: bool = True,
                 fused_residual_ln: bool = True, fused_gelu: bool = False):
        vm = model.vision_model
        self.pad_head_dim = pad_head_dim
        self.fp32_residual = fp32_residual
        # fp32 stream: each residual add + the next LayerNorm as one libeggroll pass (eggroll_resid_layernorm)
        # instead of torch's bf16->fp32 copy, add, layer_norm and bf16 cast; False keeps the torch ops (A/B)
        self.fused_residual_ln = fused_residual_ln
        self.use_kernel = use_kernel   # libeggroll's MFMA attention (eggroll_cross_attention, k = v = own tokens)
        cfg = model.config.vision_config
        self.C, self.heads = cfg.hidden_size, cfg.num_attention_heads
        self.hd = self.C // self.heads
        self.patch = cfg.patch_size
        self.act = ACT[cfg.hidden_act]
        # exact GELU in the fc1 GEMM's epilogue where fc1 runs on the 8-phase kernel.  Off by default: measured
        # 1.7x SLOWER than fc1 + torch's F.gelu (842 vs 361 + 137 us per CLIP-H fc1 at the epoch's batch,
        # profiles/r12c_gelu_erf_epilogue_ab.txt) — ocml's erff is ~40 VALU ops per element and the 8-phase
        # kernel's epilogue runs at one block per CU, exposed, where torch's pass runs at full occupancy
        self.fused_gelu = fused_gelu and cfg.hidden_act == "gelu"
        emb = vm.embeddings
        self.patch_w = emb.patch_embedding.weight.detach().reshape(self.C, -1).contiguous()     # [C, 3 p p]
        self.cls = emb.class_embedding.detach()
        self.pos = emb.position_embedding.weight.detach()
        self.pre = vm.pre_layrnorm
        self.post = vm.post_layernorm
        self.proj = model.visual_projection.weight.detach()
        if fp32_residual:   # fp32 copies of the small tensors that act on the fp32 stream
            f = lambda t: t.detach().float()  # noqa: E731
            self.patch_w32, self.cls32, self.pos32, self.proj32 = f(self.patch_w), f(self.cls), f(self.pos), f(self.proj)
        self.layers: List[dict] = []
        for L in vm.encoder.layers:
            a = L.self_attn
            self.layers.append(dict(
                ln1=L.layer_norm1, ln2=L.layer_norm2,
                wqkv=torch.cat([a.q_proj.weight, a.k_proj.weight, a.v_proj.weight]).detach().contiguous(),
                bqkv=torch.cat([a.q_proj.bias, a.k_proj.bias, a.v_proj.bias]).detach().contiguous(),
                wo=a.out_proj.weight.detach(), bo=a.out_proj.bias.detach(), scale=a.scale,
                w1=L.mlp.fc1.weight.detach(), b1=L.mlp.fc1.bias.detach(),
                w2=L.mlp.fc2.weight.detach(), b2=L.mlp.fc2.bias.detach()))

    @staticmethod
    def _lin(x, w, b, ours: bool):
        """x W^T + b: libeggroll's 8-phase GEMM (256x256 tile) where it measured faster than hipBLASLt —
        CLIP-H/14's q/k/v and fc1 at 128 x 257 rows, 1252 vs 1196 and 1246 vs 1169 TF/s
        (tools/dcae_gemm_probe.py ... clip, profiles/r05a_clip_gemm_hipblaslt_vs_8phase.json) — else F.linear."""
        if ours and x.dtype == torch.bfloat16 and w.shape[1] % 64 == 0:
            from . import kernels as K
            x2 = x.reshape(-1, x.shape[-1]).contiguous()
            return K.lora_linear_pop(x2, w, b, None, 0, 0, 0, 0.0, x2.shape[0], kernel=8).view(*x.shape[:-1], w.shape[0])
        return F.linear(x, w, b)

    def _fc1_act(self, y, L, ours: bool):
        """act(fc1(y)).  With fused_gelu, an exact GELU (CLIP-H/14, hidden_act "gelu") runs in the 8-phase GEMM's
        epilogue (eggroll_lora_linear_pop_epi, epi 8): the same fp32 expression and erff as torch's GELU of
        the bf16 fc1 output, so the same bits (measured slower, see __init__)."""
        if ours and self.fused_gelu and y.dtype == torch.bfloat16 and L["w1"].shape[1] % 64 == 0:
            from . import kernels as K
            y2 = y.reshape(-1, y.shape[-1]).contiguous()
            return K.lora_linear_pop_epi(y2, L["w1"], L["b1"], None, 0, 0, 0, 0.0, y2.shape[0], "gelu_erf",
                                         kernel=8).view(*y.shape[:-1], L["w1"].shape[0])
        return self.act(self._lin(y, L["w1"], L["b1"], ours))

    @staticmethod
    def _ln(mod, x):
        return F.layer_norm(x, mod.normalized_shape, mod.weight, mod.bias, mod.eps)

    @staticmethod
    def _ln32(mod, x, out_dtype):
        """LayerNorm of the fp32 stream in fp32 (the module's bf16 affine upcast), rounded once to the
        GEMM operand dtype."""
        w = None if mod.weight is None else mod.weight.float()
        b = None if mod.bias is None else mod.bias.float()
        return F.layer_norm(x, mod.normalized_shape, w, b, mod.eps).to(out_dtype)

    @torch.no_grad()
    def _forward32(self, pixels: torch.Tensor) -> torch.Tensor:
        n = pixels.shape[0]
        p, C, H, hd = self.patch, self.C, self.heads, self.hd
        dt = self.patch_w.dtype
        x = pixels.float()
        g = x.shape[-1] // p
        cols = x.view(n, 3, g, p, g, p).permute(0, 2, 4, 1, 3, 5).reshape(n, g * g, 3 * p * p)
        P = cols.shape[1]
        T = P + 1
        h = torch.empty((n, T, C), dtype=torch.float32, device=x.device)
        h[:, 0] = self.cls32
        h[:, 1:] = cols @ self.patch_w32.t()
        h += self.pos32[None, :T]
        h = F.layer_norm(h, self.pre.normalized_shape, self.pre.weight.float(), self.pre.bias.float(), self.pre.eps)
        kernel = self.use_kernel and hd in (64, 80, 112) and T <= 320
        from . import kernels as K
        last = len(self.layers) - 1
        fused = self.fused_residual_ln and dt == torch.bfloat16 and C % 8 == 0
        ln_k = lambda mod, h_, add: K.resid_layernorm_(h_, add, mod.weight, mod.bias, mod.eps)  # noqa: E731
        y_next = ln_k(self.layers[0]["ln1"], h, None) if fused else None
        big = fused and C >= 1024 and n * T >= 16384      # the CLIP-H/14 tower at the epoch's batch
        for i, L in enumerate(self.layers):
            y = y_next if fused else self._ln32(L["ln1"], h, dt)
            last_i = i == last
            if kernel:
                qkv = self._lin(y, L["wqkv"], L["bqkv"], big).view(n * T, 3 * C)
                qv = qkv[::T] if last_i else qkv
                o = K.cross_attention(qv, qkv[:, C:], qkv[:, 2 * C:], n, 1 if last_i else T, H, hd, T, L["scale"])
                o = o.view(n, -1, C)
            else:
                qkv = F.linear(y, L["wqkv"], L["bqkv"]).view(n, T, 3, H, hd)
                k, v = qkv[:, :, 1].transpose(1, 2), qkv[:, :, 2].transpose(1, 2)
                q = (qkv[:, :1, 0] if last_i else qkv[:, :, 0]).transpose(1, 2)
                o = F.scaled_dot_product_attention(q, k, v, scale=L["scale"]).transpose(1, 2).reshape(n, -1, C)
            if last_i:       # only the [CLS] row is read by get_image_features
                h = h[:, :1]
            if fused:        # h += out_proj(o); y = LN2(h)  (h: [n, T, C], or the [CLS] rows [n, 1, C] strided)
                h2 = h.view(n * T, C) if not last_i else h[:, 0]
                y = ln_k(L["ln2"], h2, F.linear(o.reshape(-1, C), L["wo"], L["bo"]))
                m = F.linear(self._fc1_act(y, L, big and not last_i), L["w2"], L["b2"])
                if not last_i:   # h += mlp(y); the next layer's LN1 in the same pass
                    y_next = ln_k(self.layers[i + 1]["ln1"], h2, m)
                else:
                    h = h2 + m.float()
                continue
            h = h + F.linear(o, L["wo"], L["bo"]).float()
            y = self._ln32(L["ln2"], h, dt)
            h = h + F.linear(self.act(F.linear(y, L["w1"], L["b1"])), L["w2"], L["b2"]).float()
        hc = h if h.dim() == 2 else h[:, 0]
        pooled = F.layer_norm(hc, self.post.normalized_shape, self.post.weight.float(), self.post.bias.float(),
                              self.post.eps)
        return pooled @ self.proj32.t()

    @torch.no_grad()
    def __call__(self, pixels: torch.Tensor) -> torch.Tensor:
        """pixels [n, 3, S, S] (normalised fp32) -> projected image embeddings [n, proj] fp32."""
        if self.fp32_residual:
            return self._forward32(pixels)
        n = pixels.shape[0]
        p, C, H, hd = self.patch, self.C, self.heads, self.hd
        x = pixels.to(self.patch_w.dtype)
        g = x.shape[-1] // p                                                    # non-overlapping patches:
        cols = x.view(n, 3, g, p, g, p).permute(0, 2, 4, 1, 3, 5).reshape(n, g * g, 3 * p * p)  # (c, ky, kx)
        P = cols.shape[1]
        tok = torch.empty((n, P + 1, C), dtype=x.dtype, device=x.device)
        tok[:, 0] = self.cls
        tok[:, 1:] = cols @ self.patch_w.t()
        tok += self.pos[None, :P + 1]
        h = self._ln(self.pre, tok)
        T = P + 1
        last = len(self.layers) - 1
        for i, L in enumerate(self.layers):
            y = self._ln(L["ln1"], h)
            if self.use_kernel and hd in (64, 80, 112) and T <= 320:
                from . import kernels as K
                qkv = F.linear(y, L["wqkv"], L["bqkv"]).view(n * T, 3 * C)
                last_i = i == len(self.layers) - 1
                # self-attention as the caption-attention kernel with the image's own tokens as keys; on the
                # last layer only the [CLS] query rows (row stride T) are attended
                qv = qkv[::T] if last_i else qkv
                o = K.cross_attention(qv, qkv[:, C:], qkv[:, 2 * C:], n, 1 if last_i else T, H, hd, T, L["scale"])
                if last_i:
                    h = h[:, :1]
                h = h + F.linear(o.view(n, -1, C), L["wo"], L["bo"])
                y = self._ln(L["ln2"], h)
                h = h + F.linear(self.act(F.linear(y, L["w1"], L["b1"])), L["w2"], L["b2"])
                continue
            qkv = F.linear(y, L["wqkv"], L["bqkv"]).view(n, T, 3, H, hd)
            k, v = qkv[:, :, 1].transpose(1, 2), qkv[:, :, 2].transpose(1, 2)
            if i == last:           # only the [CLS] row is read by get_image_features
                q = qkv[:, :1, 0].transpose(1, 2)
                h = h[:, :1]
            else:
                q = qkv[:, :, 0].transpose(1, 2)
            pad = (-hd) % 64 if self.pad_head_dim else 0
            if pad:   # zero-padded head dims: exact (zeros in q.k, zero output columns); measured slower at 80
                q, k, v = (F.pad(t, (0, pad)) for t in (q, k, v))
            o = F.scaled_dot_product_attention(q, k, v, scale=L["scale"])
            if pad:
                o = o[..., :hd]
            o = o.transpose(1, 2).reshape(n, -1, C)
            h = h + F.linear(o, L["wo"], L["bo"])
            y = self._ln(L["ln2"], h)
            h = h + F.linear(self.act(F.linear(y, L["w1"], L["b1"])), L["w2"], L["b2"])
        pooled = self._ln(self.post, h[:, 0])
        return F.linear(pooled, self.proj).float()
