"""InfinityES (models/Infinity.py:29-556) on the MI355X build: the Infinity bitwise-AR generation the
ES epoch of BASELINE configs[4] evaluates, member-batched.

Reference semantics kept: prompts arrive as per-prompt "compact" T5 features [L_i, 2048] with their
lengths (models/Infinity.py:257-335, 362-388); one call generates all images of a list with per-scale
cfg / tau lists (a scalar repeats, a short list pads with its last value, a long one truncates:
models/Infinity.py:463-489); every call seeds its sampling generator with `seed`; images come back
as PIL after Infinity's `(img + 1) / 2 * 255 -> uint8` and the channel flip.  The text encoder
(flan-t5-xl) is not available offline: prompts come from an encoded file or the synthetic set.
Knobs the reference passes through to Infinity that change sampling beyond top-k / top-p (gumbel,
cfg_exp_k, softmax_merge_topk, gt_leak, sampling_per_bits > 1, negative prompts, a non-zero
cfg_insertion_layer) raise NotImplementedError instead of being ignored.
"""
from __future__ import annotations

import os
from pathlib import Path
from typing import Any, List, Optional, Sequence, Tuple, Union

import numpy as np
import torch

from .infinity import InfinityPopulationInfer, InfinityTransformer, arch_for, infinity_vae, scale_schedule
from .lora import PopulationContext, set_population


def as_schedule_list(x, name: str, T: int) -> List[float]:
    """models/Infinity.py:463-486."""
    if x is None:
        raise ValueError(f"{name} cannot be None for Infinity (need scalar or list).")
    if isinstance(x, (float, int)):
        return [float(x)] * T
    if torch.is_tensor(x):
        if x.ndim == 0:
            return [float(x.item())] * T
        x = x.detach().cpu().tolist()
    if isinstance(x, (list, tuple)):
        xs = [float(v) for v in x]
        if len(xs) < T:
            xs = xs + [xs[-1]] * (T - len(xs))
        elif len(xs) > T:
            xs = xs[:T]
        return xs
    raise TypeError(f"{name} must be float/int/tensor/list, got {type(x)}")


def images_to_uint8(images: torch.Tensor) -> torch.Tensor:
    """Infinity's postprocess on the decoder output [n, 3, H, W] (already channel-flipped): (x + 1) / 2
    * 255 in bf16, truncated to uint8 (x clamped to [-1, 1] by the decoder).  uint8-valued fp32."""
    x = images.to(torch.bfloat16)
    x = (x + 1) / 2
    return (x * 255).clamp_(0, 255).to(torch.uint8).float()


def to_pil_infinity(images: torch.Tensor) -> List[Any]:
    from PIL import Image
    arr = images_to_uint8(images).to(torch.uint8).permute(0, 2, 3, 1).cpu().numpy()
    return [Image.fromarray(a) for a in arr]


class InfinityES:
    """models/Infinity.py:29-556.  `self.transformer` (= `self.infinity`) is the LoRA target."""

    def __init__(self, *, model_path: str, text_encoder_ckpt: str, vae_path: str, vae_type: int, pn: str,
                 model_type: str = "infinity_2b", h_div_w_template: float = 1.0, text_channels: int = 2048,
                 apply_spatial_patchify: int = 0, use_flex_attn: int = 0, bf16: bool = True,
                 checkpoint_type: str = "torch", top_k: int = 900, top_p: float = 0.97, cfg_exp_k: float = 0.0,
                 gumbel: int = 0, softmax_merge_topk: int = -1, cfg_insertion_layer: int = 0,
                 sampling_per_bits: int = 1, enable_positive_prompt: int = 0, gt_leak: int = 0,
                 device: str = "cuda:0", DTYPE: torch.dtype = torch.bfloat16, sigma_data: float = 0.5,
                 # build knobs
                 synthetic_weights: bool = False, arch=None, weight_seed: int = 0, vae_chunk: int = 16,
                 kv_budget_gb: float = 120.0):
        os.environ["TOKENIZERS_PARALLELISM"] = "false"
        self.device, self.DTYPE, self.bf16 = device, torch.bfloat16, bool(bf16)
        if float(h_div_w_template) != 1.0:
            raise NotImplementedError("only the h/w = 1.0 scale templates are restated")
        self.top_k_default, self.top_p_default = int(top_k), float(top_p)
        self.cfg_exp_k_default, self.gumbel_default = float(cfg_exp_k), int(gumbel)
        self.softmax_merge_topk_default = int(softmax_merge_topk)
        self.cfg_insertion_layer_default = int(cfg_insertion_layer)
        self.sampling_per_bits_default = int(sampling_per_bits)
        self.enable_positive_prompt_default = int(enable_positive_prompt)
        self.gt_leak_default = int(gt_leak)
        self.scale_schedule = scale_schedule(pn)
        a = arch if arch is not None else arch_for(model_type, int(vae_type), int(apply_spatial_patchify),
                                                   int(text_channels))
        if arch is None and checkpoint_type not in ("torch", "torch_shard"):
            raise ValueError(f"checkpoint_type must be 'torch' or 'torch_shard', got {checkpoint_type}")
        self.arch = a
        self.vae_type = int(vae_type)
        self.text_tokenizer = self.text_encoder = None
        self.infinity = InfinityTransformer(a).to(device)
        self.vae = infinity_vae(a).to(device)
        if synthetic_weights:
            self.infinity.init_weights(weight_seed)
            self.vae.init_weights(weight_seed + 2)
            self.weights_source = "synthetic"
        else:
            # models/Infinity.py:183-235: the Infinity repo's state dict (.pth, or a shard directory with its
            # index) and the BSQ-VAE .pth, strict (checkpoints.load_infinity_transformer / load_bsq_vae_decoder)
            from . import checkpoints as ck
            for nm, pth in (("model_path", model_path), ("vae_path", vae_path)):
                if not Path(pth).exists():
                    raise FileNotFoundError(f"{nm} {pth}: no local Infinity checkpoint there (a .pth or a shard "
                                            "directory); pass synthetic_weights=True for the throughput configuration")
            ck.load_infinity_transformer(self.infinity, Path(model_path), checkpoint_type)
            ck.load_bsq_vae_decoder(self.vae, Path(vae_path))
            self.weights_source = str(model_path)
        self.transformer = self.infinity
        self.vae_chunk = int(vae_chunk)
        self.kv_budget = float(kv_budget_gb) * 2 ** 30
        self.ctx = PopulationContext()

    # ---- prompt cache (models/Infinity.py:257-349) ---------------------------------------
    def encode_prompts(self, prompts_txt_path, encoded_save_path, batch_size: int = 8, complex_human_instruction=None,
                       overwrite: bool = False, store_dtype: str = "float16"):
        enc = Path(encoded_save_path)
        if enc.is_file() and not overwrite:
            return torch.load(enc, map_location="cpu", weights_only=True)
        raise NotImplementedError("the flan-t5-xl text encoder is not available offline; provide an encoded file")

    def drop_text_encoder(self):
        self.text_encoder = None

    @staticmethod
    def _pack_compacts_for_infinity(kv_list: Sequence[torch.Tensor], lens_list: Sequence[int], device: str,
                                    kv_dtype: torch.dtype) -> Tuple[torch.Tensor, List[int], torch.Tensor, int]:
        """models/Infinity.py:361-388: (kv_compact_cat [sum L_i, C], lens, cu_seqlens_k int32 [B+1], max L)."""
        lens = [int(x) for x in lens_list]
        if len(kv_list) != len(lens):
            raise ValueError("kv_list and lens_list must have same length")
        if len(lens) == 0:
            raise ValueError("empty batch")
        cu = torch.tensor([0] + list(np.cumsum(lens).astype(np.int32)), device=device, dtype=torch.int32)
        kv_cat = torch.cat([kv.to(device=device, dtype=kv_dtype) for kv in kv_list], dim=0)
        return kv_cat, lens, cu, int(max(lens))

    def _check_knobs(self, cfg_exp_k, gumbel, softmax_merge_topk, gt_leak, sampling_per_bits, cfg_insertion_layer,
                     negative):
        bad = [n for n, v, ok in (("cfg_exp_k", cfg_exp_k, 0.0), ("gumbel", gumbel, 0), ("softmax_merge_topk",
                                  softmax_merge_topk, -1), ("gt_leak", gt_leak, 0), ("sampling_per_bits",
                                  sampling_per_bits, 1), ("cfg_insertion_layer", cfg_insertion_layer, 0)) if v != ok]
        if negative:
            bad.append("negative prompts")
        if bad:
            raise NotImplementedError(f"Infinity sampling knobs not built: {bad}")

    def _distinct(self, kv_list, lens_list):
        """Distinct prompts (by tensor identity + length) -> (kv list, lens, image -> distinct index)."""
        keys, kvs, lens, idx = {}, [], [], []
        for kv, L in zip(kv_list, lens_list):
            key = (kv.data_ptr(), int(L), tuple(kv.shape))
            if key not in keys:
                keys[key] = len(kvs)
                kvs.append(kv.to(self.device))
                lens.append(int(L))
            idx.append(keys[key])
        return kvs, lens, torch.tensor(idx, device=self.device)

    def members_per_pass(self, n: int, B: int) -> int:
        """Members per generation pass so the per-block KV caches stay within kv_budget."""
        a = self.arch
        ltot = sum(h * w for _, h, w in self.scale_schedule)
        per_member = a.depth * 2 * (2 * B) * ltot * a.C * 2
        return max(1, min(n, int(self.kv_budget // max(per_member, 1))))

    def _decode(self, summed: torch.Tensor) -> torch.Tensor:
        outs = [self.vae(summed[s:s + self.vae_chunk]).clamp_(-1, 1).flip(1)
                for s in range(0, summed.shape[0], self.vae_chunk)]
        return torch.cat(outs)

    @torch.no_grad()
    def _generate(self, kvs, lens, idx, n: int, seed: int, cfg_list, tau_list, top_k, top_p, micro_batch: int,
                  theta_pop: Optional[torch.Tensor], force_bits=None, keep_logits: bool = False):
        T = len(self.scale_schedule)
        cfg = as_schedule_list(cfg_list, "cfg_list", T)
        tau = as_schedule_list(tau_list, "tau_list", T)
        inf = InfinityPopulationInfer(self.transformer, self.vae)
        B = int(idx.numel())
        per = self.members_per_pass(n, B) if theta_pop is not None else 1
        imgs, extras = [], []
        for k0 in range(0, n, per):
            k1 = min(n, k0 + per)
            if theta_pop is not None:
                self.ctx.theta_pop, self.ctx.n_members = theta_pop[k0:k1], k1 - k0
                set_population(self.transformer, self.ctx)
            try:
                fb = None if force_bits is None else [f.view(n, B, *f.shape[1:])[k0:k1].reshape(-1, *f.shape[1:])
                                                      for f in force_bits]
                summed, bits, logits = inf.run(kvs, lens, idx, k1 - k0, self.scale_schedule, seed, cfg, tau, top_k,
                                               top_p, micro_batch, fb, keep_logits)
            finally:
                if theta_pop is not None:
                    set_population(self.transformer, None)
                    self.ctx.theta_pop = None
            imgs.append(self._decode(summed))
            extras.append((bits, logits))
        self.last_bits = [torch.cat([e[0][s] for e in extras]) for s in range(T)]
        self.last_logits = [torch.cat([e[1][s] for e in extras]) for s in range(T)] if keep_logits else []
        return torch.cat(imgs)

    # ---- reference API (single member: the transformer's own LoRA params) -----------------
    @torch.no_grad()
    def generate_one_batch_from_compacts(self, *, kv_compact_list: Sequence[torch.Tensor], lens_list: Sequence[int],
                                         seed: int, guidance_scale: float, cfg_list: Union[float, List[float]],
                                         tau_list: Union[float, List[float]], negative_kv_compact_list=None,
                                         negative_lens_list=None, top_k: Optional[int] = None,
                                         top_p: Optional[float] = None, cfg_exp_k: Optional[float] = None,
                                         cfg_insertion_layer: Optional[int] = None, vae_type: Optional[int] = None,
                                         sampling_per_bits: Optional[int] = None, gumbel: Optional[int] = None,
                                         softmax_merge_topk: Optional[int] = None, gt_leak: Optional[int] = None,
                                         gt_ls_Bl: Any = None, output_type: str = "pil", micro_batch: int = 0):
        """models/Infinity.py:413-539: one call for the whole list (B = len(kv_compact_list)).  The
        per-scale CFG weights are cfg_list (guidance_scale is the reference's cfg_sc, which the
        per-scale list supersedes)."""
        B = int(len(lens_list))
        if B == 0:
            return []
        self._check_knobs(self.cfg_exp_k_default if cfg_exp_k is None else cfg_exp_k,
                          self.gumbel_default if gumbel is None else gumbel,
                          self.softmax_merge_topk_default if softmax_merge_topk is None else softmax_merge_topk,
                          self.gt_leak_default if gt_leak is None else gt_leak,
                          self.sampling_per_bits_default if sampling_per_bits is None else sampling_per_bits,
                          self.cfg_insertion_layer_default if cfg_insertion_layer is None else cfg_insertion_layer,
                          negative_kv_compact_list is not None and negative_lens_list is not None)
        if vae_type is not None and int(vae_type) != self.vae_type:
            raise ValueError(f"vae_type {vae_type} differs from the loaded VAE's {self.vae_type}")
        if len(kv_compact_list) != B:
            raise ValueError("kv_list and lens_list must have same length")
        set_population(self.transformer, None)
        kvs, lens, idx = self._distinct(kv_compact_list, lens_list)
        imgs = self._generate(kvs, lens, idx, 1, seed, cfg_list, tau_list,
                              self.top_k_default if top_k is None else int(top_k),
                              self.top_p_default if top_p is None else float(top_p), micro_batch, None)
        return imgs if output_type == "pt" else to_pil_infinity(imgs)

    def generate(self, prompt_embeds=None, prompt_attention_mask=None, latents=None, seed: int = 0,
                 guidance_scale: float = 3.0, width_latent: int = 32, height_latent: int = 32, **kwargs):
        raise NotImplementedError("Use InfinityBackend.generate_flat(...) which indexes prompt cache and calls "
                                  "generate_one_batch_from_compacts().")

    # ---- engine API --------------------------------------------------------------------
    @torch.no_grad()
    def generate_population(self, kv_list: Sequence[torch.Tensor], lens_list: Sequence[int],
                            prompt_index: torch.Tensor, theta_pop: torch.Tensor, seed: int, cfg_list, tau_list,
                            top_k: int, top_p: float, micro_batch: int = 0, force_bits=None,
                            keep_logits: bool = False) -> torch.Tensor:
        """All members of theta_pop [n, D]: kv_list / lens_list = the DISTINCT prompts, prompt_index [B]
        image -> distinct prompt.  Returns images [n*B, 3, H, W] in [-1, 1] (member-major, channel order
        as the reference's PIL images)."""
        kvs = [kv.to(self.device) for kv in kv_list]
        return self._generate(kvs, [int(v) for v in lens_list], prompt_index.to(self.device), int(theta_pop.shape[0]),
                              seed, cfg_list, tau_list, top_k, top_p, micro_batch, theta_pop, force_bits, keep_logits)
