"""Sana-Sprint one-step generator (models/SanaSprint.py:10-164 `SanaOneStep`), ES-compatible
(models/baseEGG.py:14-77 `ESBaseModel` contract: `self.transformer` is the LoRA target,
`generate(...) -> (images, latents_out)`), plus the population entry point that evaluates every
local member in one batched forward.

One-step SCM / trigflow math exactly as the reference (models/SanaSprint.py:78-164):
  latents = randn(b, 32, h, w, Generator(device).manual_seed(seed), dtype=DTYPE) * sigma_data
  scm = sin(1.571) / (cos(1.571) + sin(1.571));  guidance = g * guidance_embeds_scale
  eps = nan_to_num(transformer(latents / sigma_data, scm, prompt, mask, guidance))
  pred = ((1-2s) x + (1-2s+2s^2) eps) / sqrt(s^2 + (1-s)^2) * sigma_data
  x0 = (0.267 latents - 0.964 pred) / sigma_data;  image = vae.decode(x0 / scaling_factor)
Common random numbers: every member uses the same latents (seed = epoch) and prompts
(unifed_es.py:163), so latents are drawn once and broadcast over members.
"""
from __future__ import annotations

import math
from pathlib import Path
from typing import Any, List, Optional

import torch

from .dcae import DCAEDecoder
from .lora import PopulationContext, set_population
from .sana import SANA_SPRINT_1_6B, SanaArch, SanaTransformer2DModel


class ESBaseModel:
    """models/baseEGG.py:14-77."""

    def __init__(self, model_name: str, device: str = "cuda:0", DTYPE: torch.dtype = torch.float32,
                 sigma_data: float = 0.5):
        self.model_name = str(model_name)
        self.device = str(device)
        self.DTYPE = DTYPE
        self.sigma_data = float(sigma_data)
        self.transformer: Optional[torch.nn.Module] = None

    def generate(self, *a, **k):
        raise NotImplementedError("Subclasses must implement generate()")

    def encode_prompts(self, *a, **k):
        raise NotImplementedError("Subclasses must implement encode_prompts()")


class SanaOneStep(ESBaseModel):
    """models/SanaSprint.py:10-60.  Weights: `model_name` is a LOCAL diffusers-format directory
    (transformer/ + vae/, loaded by checkpoints.py; the architecture comes from its config.json files,
    `arch` / `vae_*` are ignored), or — only with synthetic_weights=True — anything, in which case
    the given architecture is built with seeded synthetic weights (throughput runs).
    Anything else raises FileNotFoundError: there is no hub access, and silently substituting random
    weights for a named checkpoint would produce plausible-looking but meaningless numbers."""

    def __init__(self, model_name: str = "Efficient-Large-Model/Sana_Sprint_1.6B_1024px_diffusers",
                 device: str = "cuda:0", DTYPE: torch.dtype = torch.float16, sigma_data: float = 0.5,
                 arch: SanaArch = SANA_SPRINT_1_6B, vae_widths=(128, 256, 512, 512, 1024, 1024),
                 vae_layers=(3, 3, 3, 3, 3, 3), weight_seed: int = 0, vae_chunk: int = 8,
                 synthetic_weights: bool = False):
        from . import checkpoints as C
        super().__init__(model_name, device, DTYPE, sigma_data)
        dev = torch.device(device)
        root = Path(str(model_name))
        if C.is_local_model_dir(str(model_name)):
            arch = C.sana_arch_from_config(C.read_config(root / "transformer"))
            vkw = C.dcae_build_kwargs(C.read_config(root / "vae"))
            with torch.device(dev):
                self.transformer = SanaTransformer2DModel(arch)
                self.vae = DCAEDecoder(**vkw)
            C.load_sana_transformer(self.transformer, root / "transformer")
            C.load_dcae_decoder(self.vae, root / "vae")
            self.weights_source = str(root)
        elif synthetic_weights:
            with torch.device(dev):
                self.transformer = SanaTransformer2DModel(arch)
                self.vae = DCAEDecoder(arch.in_channels, widths=vae_widths, layers=vae_layers)
            self.transformer.init_weights(weight_seed)
            self.vae.init_weights(weight_seed + 1)
            self.weights_source = f"synthetic(seed={weight_seed})"
        else:
            why = ("exists but lacks transformer/ or vae/" if root.exists()
                   else "is not a local directory (no hub downloads offline)")
            raise FileNotFoundError(f"SanaOneStep: model_name {str(model_name)!r} {why}; pass a local diffusers "
                                    f"model directory, or synthetic_weights=True for seeded random weights")
        self.transformer_config = arch
        self.vae_chunk = vae_chunk
        self.ctx = PopulationContext()

    # ---- shared one-step math -------------------------------------------------------
    def _latents(self, b: int, seed: int, h: int, w: int) -> torch.Tensor:
        g = torch.Generator(device=self.device).manual_seed(int(seed))
        lat = torch.randn(b, self.transformer_config.in_channels, h, w, device=self.device, dtype=self.DTYPE,
                          generator=g)
        return lat * self.sigma_data

    @torch.no_grad()
    def _one_step(self, latents, prompt_embeds, prompt_attention_mask, guidance_scale, reps: int,
                  prompt_index: Optional[torch.Tensor] = None):
        """prompt_index (optional): [b] image -> row of prompt_embeds / mask, which then hold the
        distinct prompts only (the images of one prompt share its caption k / v, see sana.py)."""
        b = latents.shape[0]
        lmi = latents / self.sigma_data
        t = torch.tensor(1.571, device=self.device, dtype=torch.float32)
        timestep = t.expand(b)
        scm = torch.sin(timestep) / (torch.cos(timestep) + torch.sin(timestep))
        se = scm.view(-1, 1, 1, 1)
        guidance = torch.full((b,), guidance_scale, device=self.device, dtype=self.DTYPE)
        guidance = guidance * self.transformer_config.guidance_embeds_scale

        def rep(x):
            return x if reps == 1 else x.repeat(reps, *([1] * (x.ndim - 1)))  # member-major stacking

        enc_index = None
        if prompt_index is not None:
            u = prompt_embeds.shape[0]
            enc_index = (torch.arange(reps, device=self.device)[:, None] * u + prompt_index.to(self.device)[None, :]).reshape(-1)
        eps = self.transformer(rep(lmi.float()), rep(scm.float()), rep(prompt_embeds), rep(prompt_attention_mask),
                               rep(guidance.float()), enc_index=enc_index)
        eps = torch.nan_to_num(eps.float(), nan=0.0, posinf=0.0, neginf=0.0)
        # dtype semantics of models/SanaSprint.py:138-153: eps rounded to the latent dtype (fp16) before
        # the SCM combine, which promotes to fp32 through the fp32 scm tensor; 0.267 * latents is an fp16
        # product (python scalar x fp16 tensor) before the fp32 subtraction
        eps = eps.to(self.DTYPE)
        lmi_r, se_r = rep(lmi), rep(se)
        pred = ((1 - 2 * se_r) * lmi_r + (1 - 2 * se_r + 2 * se_r ** 2) * eps) / torch.sqrt(se_r ** 2 + (1 - se_r) ** 2)
        pred = pred.float() * self.sigma_data
        x0 = (rep(0.267 * latents) - 0.964 * pred) / self.sigma_data
        z = x0 / self.vae.scaling_factor
        imgs = [self.vae(z[s:s + self.vae_chunk]) for s in range(0, z.shape[0], self.vae_chunk)]
        return torch.cat(imgs), z

    # ---- reference API (single member: the transformer's own LoRA params) ------------
    @torch.no_grad()
    def generate(self, prompt_embeds, prompt_attention_mask, latents=None, seed: int = 0, guidance_scale: float = 1.0,
                 width_latent: int = 32, height_latent: int = 32, output_type: str = "pil"):
        """models/SanaSprint.py:60-164.  Returns (images, latents in VAE scale)."""
        set_population(self.transformer, None)
        if latents is None:
            latents = self._latents(prompt_embeds.shape[0], seed, height_latent, width_latent)
        imgs, z = self._one_step(latents, prompt_embeds, prompt_attention_mask, guidance_scale, reps=1)
        if output_type == "pt":
            return imgs, z
        return to_pil(imgs), z

    # ---- engine API -----------------------------------------------------------------
    @torch.no_grad()
    def generate_population(self, prompt_embeds, prompt_attention_mask, theta_pop: torch.Tensor, seed: int,
                            guidance_scale: float, width_latent: int, height_latent: int,
                            prompt_index: Optional[torch.Tensor] = None) -> torch.Tensor:
        """All members of theta_pop [n, D] at once: returns VAE images [n*b, 3, H, W] (member-major).
        prompt_index: [b] image -> distinct-prompt row (prompt_embeds then holds the distinct prompts)."""
        n = theta_pop.shape[0]
        self.ctx.theta_pop, self.ctx.n_members = theta_pop, n
        set_population(self.transformer, self.ctx)
        try:
            b = prompt_embeds.shape[0] if prompt_index is None else prompt_index.numel()
            latents = self._latents(b, seed, height_latent, width_latent)
            imgs, _ = self._one_step(latents, prompt_embeds, prompt_attention_mask, guidance_scale, reps=n,
                                     prompt_index=prompt_index)
        finally:
            set_population(self.transformer, None)
            self.ctx.theta_pop = None
        return imgs


def to_pil(images: torch.Tensor) -> List[Any]:
    """PixArtImageProcessor.postprocess(output_type='pil')."""
    from PIL import Image
    arr = torch.round((images.float() / 2 + 0.5).clamp(0, 1) * 255).to(torch.uint8).permute(0, 2, 3, 1).cpu().numpy()
    return [Image.fromarray(a) for a in arr]
