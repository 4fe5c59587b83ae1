"""ZImageTurboES (models/zImageTurbo.py:15-407) on the MI355X build: the Z-Image-Turbo few-step
flow-matching generation the ES epoch of BASELINE configs[3] evaluates, member-batched.

Reference semantics kept: prompt embeddings are a LIST of per-prompt tensors [T_i, 2560] (the
Qwen3 hidden states ZImagePipeline.encode_prompt returns, models/zImageTurbo.py:246-296); image j of
a generate_one_batch call draws its initial latent from `torch.Generator(device).manual_seed(seed +
j)` (models/zImageTurbo.py:364-369, the per-prompt generators), [1, 16, H/8, W/8] fp32; no classifier-
free guidance at guidance_scale <= 1 (the Turbo default 0.0, unifed_es.py:416); the decoded image goes
through the PixArt-style uint8 rounding (pil_mode 0) like Sana's.  The scheduler is restated from
diffusers' FlowMatchEulerDiscreteScheduler(shift=3, 1000 train steps): sigmas linearly spaced between
the shifted sigma_max and sigma_min then shifted again, a final 0; the transformer sees t = 1 - sigma
and its output is the negated flow velocity (x_{i+1} = x_i + (sigma_{i+1} - sigma_i) * (-v)).  These
pipeline details, like the transformer, are UNPINNED (no diffusers here).

Population entry point: every member's images in one batch per step (member-major rows), the
caption path run once per distinct prompt per member (context refiner), as the Sana host does.
"""
from __future__ import annotations

from typing import Any, List, Optional, Sequence, Tuple

import numpy as np
import torch

from .flux_vae import FluxVAEDecoder
from .lora import PopulationContext, lora_modules, set_population
from .pipeline import to_pil
from .zimage import ZIMAGE_TURBO, ZImageArch, ZImageTransformer2DModel


def flow_sigmas(steps: int, shift: float = 3.0, num_train: int = 1000,
                sigma_min: Optional[float] = 0.0) -> List[float]:
    """FlowMatchEulerDiscreteScheduler(shift).set_timesteps(steps).sigmas (static shifting) as diffusers'
    ZImagePipeline calls it: the pipeline sets `scheduler.sigma_min = 0.0` before set_timesteps, so the
    unshifted grid runs linspace(1, 0, steps), is shifted, and a final 0 is appended — the last step has
    dt = 0 (a no-op update).  sigma_min=None keeps the scheduler's own default, shift(1 / num_train)."""
    sh = lambda s: shift * s / (1.0 + (shift - 1.0) * s)  # noqa: E731
    s_max = 1.0
    s_min = sh(1.0 / num_train) if sigma_min is None else float(sigma_min)
    s = np.linspace(s_max * num_train, s_min * num_train, steps) / num_train
    return [float(v) for v in sh(s)] + [0.0]


class ZImageTurboES:
    def __init__(self, model_name: str = "Tongyi-MAI/Z-Image-Turbo", device: str = "cuda:0",
                 DTYPE: torch.dtype = torch.bfloat16, num_inference_steps: int = 9, arch: ZImageArch = ZIMAGE_TURBO,
                 vae_widths: Sequence[int] = (128, 256, 512, 512), vae_chunk: int = 16, weight_seed: int = 0,
                 synthetic_weights: bool = False):
        from pathlib import Path

        from . import checkpoints as ck
        self.model_name, self.device, self.DTYPE = model_name, device, torch.bfloat16
        self.num_inference_steps = int(num_inference_steps)
        if synthetic_weights:
            self.arch = arch
            self.transformer = ZImageTransformer2DModel(arch).to(device)
            self.transformer.init_weights(weight_seed)
            self.vae = FluxVAEDecoder(widths=vae_widths).to(device)
            self.vae.init_weights(weight_seed + 2)
            self.weights_source = "synthetic"
        else:
            # ZImagePipeline.from_pretrained(model_name) (models/zImageTurbo.py:97-125): a LOCAL diffusers
            # directory (transformer/ + vae/, checkpoints.py); no hub access offline
            root = Path(model_name)
            if not (root / "transformer").is_dir() or not (root / "vae").is_dir():
                raise FileNotFoundError(f"{model_name}: not a local diffusers Z-Image directory (transformer/ + vae/); "
                                        "pass synthetic_weights=True for the throughput configuration")
            self.arch = ck.zimage_arch_from_config(ck.read_config(root / "transformer"))
            self.transformer = ZImageTransformer2DModel(self.arch).to(device)
            ck.load_zimage_transformer(self.transformer, root / "transformer")
            vk = ck.flux_vae_kwargs(ck.read_config(root / "vae"))
            vae_widths = vk["widths"]
            self.vae = FluxVAEDecoder(**vk).to(device)
            ck.load_flux_vae_decoder(self.vae, root / "vae")
            self.weights_source = str(root)
        self.vae_chunk = vae_chunk
        self.vae_scale_factor = 2 ** (len(vae_widths) - 1)
        self.ctx = PopulationContext()
        self.vae_ctx = PopulationContext()   # theta rows of the decoding members when the VAE decoder has LoRA

    # ---- helpers --------------------------------------------------------------------
    def _check_hw_divisible(self, height_px: int, width_px: int):
        div = self.vae_scale_factor * 2
        if height_px % div or width_px % div:
            raise ValueError(f"height/width must be divisible by {div}. Got height={height_px}, width={width_px}.")

    def _latents(self, n: int, seed: int, height_px: int, width_px: int) -> torch.Tensor:
        """Image j: Generator(seed + j), [16, H/8, W/8] fp32 (the per-prompt generators)."""
        h, w = height_px // self.vae_scale_factor, width_px // self.vae_scale_factor
        out = []
        for j in range(n):
            g = torch.Generator(device=self.device).manual_seed(int(seed) + j)
            out.append(torch.randn(1, self.arch.in_channels, h, w, device=self.device, dtype=torch.float32, generator=g))
        return torch.cat(out)

    def _captions(self, embeds: Sequence[torch.Tensor]) -> Tuple[torch.Tensor, torch.Tensor]:
        """Distinct prompt embeddings -> [U, Lc, cap_dim] bf16 (zero beyond each caption; Lc = the longest
        caption rounded up to seq_multiple) and the captions' own token counts [U] (the model pads each
        to a multiple of seq_multiple with its cap_pad_token)."""
        m = self.arch.seq_multiple
        real = [int(e.shape[0]) for e in embeds]
        Lc = max(-(-r // m) * m for r in real)
        cap = torch.zeros(len(embeds), Lc, self.arch.cap_feat_dim, device=self.device, dtype=torch.bfloat16)
        for u, e in enumerate(embeds):
            cap[u, :e.shape[0]] = e.to(self.device, torch.bfloat16)
        return cap, torch.tensor(real, device=self.device)

    @torch.no_grad()
    def _sample(self, lat: torch.Tensor, cap: torch.Tensor, cap_lens: torch.Tensor, prompt_index: torch.Tensor,
                n_rep: int, steps: int) -> torch.Tensor:
        sig = flow_sigmas(steps)
        capr = cap.repeat(n_rep, 1, 1) if n_rep > 1 else cap
        x = lat.repeat(n_rep, 1, 1, 1) if n_rep > 1 else lat
        for i in range(steps):
            t = torch.full((1,), 1.0 - sig[i], device=self.device, dtype=torch.float32)
            v = self.transformer(x, t, capr, cap_lens, prompt_index, n_rep=n_rep)
            x = x + (sig[i + 1] - sig[i]) * (-v)
        z = x / self.vae.scaling_factor + self.vae.shift_factor
        if self.vae_ctx.theta_pop is None:
            return torch.cat([self.vae(z[s:s + self.vae_chunk]) for s in range(0, z.shape[0], self.vae_chunk)])
        # VAE-decoder LoRA on a population: every decode chunk holds whole members or a slice of one member,
        # and the decoder's LoRA'd linears see exactly those members' theta rows
        tp, b = self.vae_ctx.theta_pop, z.shape[0] // n_rep
        out = []
        if b <= self.vae_chunk:
            per = max(1, self.vae_chunk // b)
            for k0 in range(0, n_rep, per):
                k1 = min(n_rep, k0 + per)
                out.append(self._decode_members(z[k0 * b:k1 * b], tp[k0:k1]))
        else:
            for k in range(n_rep):
                for s in range(0, b, self.vae_chunk):
                    out.append(self._decode_members(z[k * b + s:k * b + min(b, s + self.vae_chunk)], tp[k:k + 1]))
        return torch.cat(out)

    def _decode_members(self, z: torch.Tensor, theta_rows: torch.Tensor) -> torch.Tensor:
        sub = PopulationContext()
        sub.theta_pop, sub.n_members = theta_rows, theta_rows.shape[0]
        set_population(self.vae, sub)
        try:
            return self.vae(z)
        finally:
            set_population(self.vae, None)

    # ---- reference API (single member: the transformer's own LoRA params) ------------
    @torch.no_grad()
    def generate_one_batch(self, prompt_embeds: List[torch.Tensor], seed: int = 0, guidance_scale: float = 0.0,
                           width_px: int = 384, height_px: int = 384, num_inference_steps: Optional[int] = None,
                           micro_batch: int = 1, max_sequence_length: int = 512, output_type: str = "pil"):
        """models/zImageTurbo.py:339-407: images for a list of prompt embeddings (micro_batch only chunks
        the reference's pipeline calls; the latents are per-image, so it does not change the result)."""
        if guidance_scale > 1.0:
            raise NotImplementedError("classifier-free guidance (guidance_scale > 1) is not built; Turbo uses 0.0")
        self._check_hw_divisible(height_px, width_px)
        steps = self.num_inference_steps if num_inference_steps is None else int(num_inference_steps)
        set_population(self.transformer, None)
        embeds = [e[:max_sequence_length] for e in prompt_embeds]
        cap, lens = self._captions(embeds)
        idx = torch.arange(len(embeds), device=self.device)
        imgs = self._sample(self._latents(len(embeds), seed, height_px, width_px), cap, lens, idx, 1, steps)
        return (imgs if output_type == "pt" else to_pil(imgs)), None

    def generate(self, prompt_embeds, prompt_attention_mask=None, latents=None, seed: int = 0,
                 guidance_scale: float = 0.0, width_latent: int = 32, height_latent: int = 32, width_px: int = 1024,
                 height_px: int = 1024, num_inference_steps: Optional[int] = None):
        """models/zImageTurbo.py:313-337 (width_latent / height_latent unused, as there)."""
        return self.generate_one_batch(prompt_embeds, seed=seed, guidance_scale=guidance_scale, width_px=width_px,
                                       height_px=height_px, num_inference_steps=num_inference_steps)

    # ---- engine API -----------------------------------------------------------------
    @torch.no_grad()
    def generate_population(self, prompt_embeds: Sequence[torch.Tensor], prompt_index: torch.Tensor,
                            theta_pop: torch.Tensor, seed: int, guidance_scale: float, width_px: int, height_px: int,
                            num_inference_steps: Optional[int] = None) -> torch.Tensor:
        """All members of theta_pop [n, D] at once: prompt_embeds = the DISTINCT prompts, prompt_index [b]
        image -> distinct prompt.  Returns decoded images [n*b, 3, H, W] (member-major)."""
        if guidance_scale > 1.0:
            raise NotImplementedError("classifier-free guidance (guidance_scale > 1) is not built; Turbo uses 0.0")
        self._check_hw_divisible(height_px, width_px)
        steps = self.num_inference_steps if num_inference_steps is None else int(num_inference_steps)
        n = theta_pop.shape[0]
        self.ctx.theta_pop, self.ctx.n_members = theta_pop, n
        set_population(self.transformer, self.ctx)
        if any(True for _ in lora_modules(self.vae)):
            self.vae_ctx.theta_pop, self.vae_ctx.n_members = theta_pop, n
        try:
            cap, lens = self._captions(prompt_embeds)
            b = prompt_index.numel()
            return self._sample(self._latents(b, seed, height_px, width_px), cap, lens, prompt_index.to(self.device),
                                n, steps)
        finally:
            set_population(self.transformer, None)
            self.ctx.theta_pop = None
            self.vae_ctx.theta_pop = None
