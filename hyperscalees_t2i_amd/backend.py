"""ES backend interface and the Sana one-step backend (es_backend.py:16-292), MI355X edition.

Same duck-typed surface as the reference (`init_and_attach_lora`, `compile_if_requested`,
`collect_lora_params`, `save_lora`, `step_sampling_info`, `generate_flat`) so a
unifed_es.py-shaped driver runs unchanged, plus the population entry point
`generate_population(flat_ids, seed, guidance_scale, theta_pop)` that evaluates all local
members in one batched forward (the reference loops over members, unifed_es.py:159-163).
Errors are Python exceptions as in the reference (FileNotFoundError / RuntimeError / ValueError).
"""
from __future__ import annotations

import json
from dataclasses import dataclass, field
from pathlib import Path
from typing import Any, Callable, Dict, List, Optional, Sequence, Tuple, Union

import torch

from .es import get_trainable_params_and_shapes, repeat_batches, sample_classes_unique, sample_indices_unique
from .lora import lora_modules
from .pipeline import SanaOneStep
from .sana import SANA_LORA_TARGETS, SANA_SPRINT_1_6B, SanaArch, attach_lora
from .var import VAR_LORA_TARGETS, VARArch, VARClassGenerator


class ESBackend:
    """es_backend.py:16-57."""

    name: str

    def init_and_attach_lora(self) -> None:
        raise NotImplementedError

    def compile_if_requested(self) -> None:
        pass

    def collect_lora_params(self) -> Tuple[List[torch.nn.Parameter], List[Tuple[int, ...]]]:
        raise NotImplementedError

    def save_lora(self, save_dir: Path) -> None:
        raise NotImplementedError

    def step_sampling_info(self, seed: int) -> Dict[str, Any]:
        raise NotImplementedError

    def generate_flat(self, flat_ids: List[int], seed: int, guidance_scale: float,
                      flat_seeds: Optional[List[int]] = None) -> List[Any]:
        """es_backend.py:51-57: images for each flat_id in order; flat_seeds: optional per-image
        deterministic seeds (same length as flat_ids)."""
        raise NotImplementedError

    def generate_population(self, flat_ids: List[int], seed: int, guidance_scale: float,
                            theta_pop: torch.Tensor) -> torch.Tensor:
        raise NotImplementedError

    def members_per_pass(self) -> Optional[int]:
        """Largest number of members one generate_population call evaluates (ESEngine splits a rank's
        members into passes of this size, fixed boundaries from member 0); None = all in one pass."""
        return None


@dataclass
class SanaConfig:
    """es_backend.py:64-93 (+ synthetic-data / architecture knobs of this build)."""

    model_name: str = "Efficient-Large-Model/Sana_Sprint_1.6B_1024px_diffusers"
    backend_mode: str = "one_step"
    prompts_txt_path: str = "prompts_train"
    encoded_prompt_path: str = ""
    auto_encode_if_missing: bool = False
    encode_batch_size: int = 8
    guidance_scale: float = 4.5
    width_latent: int = 32            # 32 -> 1024 px (BASELINE configs); reference CLI default 16 -> 512 px
    height_latent: int = 32
    batch_size: int = 1
    prompts_per_gen: int = 4
    batches_per_gen: int = 4
    max_log_batches: int = 1
    torch_compile: bool = False
    compile_mode: str = "max-autotune"
    compile_fullgraph: bool = True
    dtype_latents: str = "float16"
    lora_r: int = 2
    lora_alpha: int = 8
    lora_dropout: float = 0.0
    lora_target_modules: List[str] = field(default_factory=lambda: list(SANA_LORA_TARGETS))
    # build-specific
    arch: SanaArch = field(default_factory=lambda: SANA_SPRINT_1_6B)
    vae_widths: Tuple[int, ...] = (128, 256, 512, 512, 1024, 1024)
    vae_layers: Tuple[int, ...] = (3, 3, 3, 3, 3, 3)
    vae_chunk: int = 8
    # members per population pass (ESEngine): 8 keeps every GEMM operand of the 1024-px forward under the
    # 32-bit buffer range (the FFN's 16-image x 1024-token x 5632 hidden map is 184 MB per member: 11
    # members reach 2 GiB) and fixes the batch a member is evaluated in: passes sit on global member
    # indices (ESEngine.member_passes), so theta' does not depend on how many ranks share the population
    # when every shard boundary is a multiple of it (configs[2]: 8 ranks x 8 == one process x 64)
    members_per_pass: int = 8
    synthetic_prompts: int = 4        # used when encoded_prompt_path is empty
    lora_b_std: float = 0.02          # nonzero B so the LoRA path is live
    lora_seed: int = 1234
    weight_seed: int = 0
    # model_name must be a local diffusers directory (transformer/ + vae/, checkpoints.py); True builds
    # `arch` with seeded synthetic weights instead (the benchmark's throughput configuration)
    synthetic_weights: bool = False


def synthetic_prompt_data(P: int = 4, seq: int = 300, dim: int = 2304, seed: int = 0) -> Dict[str, Any]:
    """Same dict format as encode_prompts_from_txt.py / SanaOneStep.encode_prompts:
    prompts, prompt_embeds [P, 300, 2304] fp16, prompt_attention_mask [P, 300] (lengths U[8, 300])."""
    g = torch.Generator().manual_seed(seed)
    emb = torch.randn(P, seq, dim, generator=g).to(torch.float16)
    lens = torch.randint(8, seq + 1, (P,), generator=g)
    mask = (torch.arange(seq)[None, :] < lens[:, None]).to(torch.int64)
    prompts = [f"synthetic prompt {i}: a detailed photo of object {i}" for i in range(P)]
    return {"prompts": prompts, "prompt_embeds": emb, "prompt_attention_mask": mask}


class SanaBackend(ESBackend):
    def __init__(self, device: str, cfg: SanaConfig):
        if cfg.backend_mode != "one_step":
            raise ValueError(f"Unknown/unsupported Sana backend_mode: {cfg.backend_mode} (one_step only)")
        self.name = f"sana_{cfg.backend_mode}"
        self.device = device
        self.cfg = cfg
        self.es_model: Optional[SanaOneStep] = None
        self.prompt_data = None
        self.base_prompt_embeds = None
        self.base_attention_mask = None
        self.prompts_list = None
        self._dev_prompts = None

    def _dtype(self) -> torch.dtype:
        return torch.bfloat16 if self.cfg.dtype_latents.lower() == "bfloat16" else torch.float16

    def _load_or_encode_prompts(self):
        """es_backend.py:112-170.  Loads with weights_only=True; no text encoder offline."""
        if self.cfg.encoded_prompt_path:
            enc = Path(self.cfg.encoded_prompt_path)
            if not enc.is_file():
                raise FileNotFoundError(f"encoded_prompt_path not found and auto_encode unsupported: {enc}")
            self.prompt_data = torch.load(enc, map_location="cpu", weights_only=True)
        else:
            self.prompt_data = synthetic_prompt_data(self.cfg.synthetic_prompts)
        self.base_prompt_embeds = self.prompt_data["prompt_embeds"]
        self.base_attention_mask = self.prompt_data["prompt_attention_mask"]
        self.prompts_list = self.prompt_data.get("prompts", None)
        if not torch.is_tensor(self.base_prompt_embeds):
            raise RuntimeError("Sana expects prompt_embeds as a Tensor [P, seq, dim].")
        if not torch.is_tensor(self.base_attention_mask):
            raise RuntimeError("Sana expects prompt_attention_mask as a Tensor [P, seq].")
        self._dev_prompts = (self.base_prompt_embeds.to(self.device), self.base_attention_mask.to(self.device))

    def init_and_attach_lora(self):
        self._load_or_encode_prompts()
        c = self.cfg
        self.es_model = SanaOneStep(c.model_name, device=self.device, DTYPE=self._dtype(), sigma_data=0.5, arch=c.arch,
                                    vae_widths=c.vae_widths, vae_layers=c.vae_layers, weight_seed=c.weight_seed,
                                    vae_chunk=c.vae_chunk, synthetic_weights=c.synthetic_weights)
        n = attach_lora(self.es_model.transformer, c.lora_r, c.lora_alpha, c.lora_target_modules)
        if n == 0:
            raise RuntimeError("no LoRA target module matched")
        g = torch.Generator(device=self.device).manual_seed(c.lora_seed)
        for m in lora_modules(self.es_model.transformer):
            m.reset_lora(g, b_std=c.lora_b_std)
        self.es_model.transformer.eval()

    def collect_lora_params(self):
        return get_trainable_params_and_shapes(self.es_model.transformer)

    def save_lora(self, save_dir: Path) -> None:
        """PEFT-style adapter dir: adapter_config.json + adapter_model.safetensors
        (keys base_model.model.<module>.lora_{A,B}.weight)."""
        _save_adapter(self.es_model.transformer, Path(save_dir),
                      {"peft_type": "LORA", "r": self.cfg.lora_r, "lora_alpha": self.cfg.lora_alpha,
                       "lora_dropout": self.cfg.lora_dropout, "target_modules": list(self.cfg.lora_target_modules),
                       "base_model_name_or_path": self.cfg.model_name, "bias": "none", "task_type": None})

    def load_lora(self, save_dir: Path) -> None:
        """Inverse of save_lora (resume; the reference is write-only), see _load_adapter."""
        _load_adapter(self.es_model.transformer, Path(save_dir))

    def step_sampling_info(self, seed: int) -> Dict[str, Any]:
        """es_backend.py:234-263 (bit-exact indices: np.random.RandomState(seed).choice)."""
        P = int(self.base_prompt_embeds.shape[0])
        unique_ids = sample_indices_unique(seed=seed, total=P, k=self.cfg.prompts_per_gen)
        flat_ids = repeat_batches(unique_ids, repeats=self.cfg.batches_per_gen)
        pid_to_j = {pid: j for j, pid in enumerate(unique_ids)}
        m = len(unique_ids)
        name = (lambda pid: self.prompts_list[pid] if self.prompts_list is not None else f"prompt_{pid}")
        log_batches = int(max(0, min(self.cfg.max_log_batches, self.cfg.batches_per_gen)))
        return dict(unique_ids=unique_ids, flat_ids=flat_ids, unique_texts=[name(p) for p in unique_ids],
                    flat_texts=[name(p) for p in flat_ids], pid_to_j=pid_to_j, m=m,
                    total_imgs_per_indiv=len(flat_ids), total_imgs_for_logging=log_batches * m,
                    log_batches=log_batches)

    def _gather(self, flat_ids):
        pe, am = self._dev_prompts
        idx = torch.as_tensor(flat_ids, device=pe.device)
        return pe.index_select(0, idx), am.index_select(0, idx)

    def generate_flat(self, flat_ids: List[int], seed: int, guidance_scale: float,
                      flat_seeds: Optional[List[int]] = None) -> List[Any]:
        """es_backend.py:265-292: one member (the transformer's current LoRA params), PIL images.
        flat_seeds (es_backend.py:51-57): image i draws its latents from Generator(seed=flat_seeds[i])
        instead of all images sharing one batched draw from `seed`."""
        pe, am = self._gather(flat_ids)
        latents = None
        if flat_seeds is not None:
            if len(flat_seeds) != len(flat_ids):
                raise ValueError(f"flat_seeds has {len(flat_seeds)} entries, flat_ids {len(flat_ids)}")
            m = self.es_model
            latents = torch.cat([m._latents(1, int(s), self.cfg.height_latent, self.cfg.width_latent)
                                 for s in flat_seeds])
        images, _ = self.es_model.generate(prompt_embeds=pe, prompt_attention_mask=am, latents=latents, seed=seed,
                                           guidance_scale=guidance_scale, width_latent=self.cfg.width_latent,
                                           height_latent=self.cfg.height_latent)
        return images

    def generate_population(self, flat_ids: List[int], seed: int, guidance_scale: float,
                            theta_pop: torch.Tensor) -> torch.Tensor:
        """flat_ids repeats each sampled prompt batches_per_gen times (repeat_batches): the distinct
        prompts are gathered once and every image points at its prompt's row, so the caption path
        (caption projection, to_k / to_v of every block) runs on m instead of m*R captions per member."""
        uniq = list(dict.fromkeys(int(f) for f in flat_ids))
        idx = torch.tensor([uniq.index(int(f)) for f in flat_ids], device=self.device)
        pe, am = self._gather(uniq)
        return self.es_model.generate_population(pe, am, theta_pop, seed, guidance_scale, self.cfg.width_latent,
                                                 self.cfg.height_latent, prompt_index=idx)

    def members_per_pass(self) -> Optional[int]:
        return self.cfg.members_per_pass or None


# ---------------------------------------------------------------------------------------
# VAR backend (es_backend.py:299-450) — BASELINE configs[0]
# ---------------------------------------------------------------------------------------


def _adapter_keys(model: torch.nn.Module, rename: Optional[Callable[[str], str]] = None) -> Dict[str, torch.Tensor]:
    """PEFT save_pretrained key names of the model's trainable (LoRA) parameters: base_model.model.<name>,
    <name> the wrapped module's own parameter name (`rename` maps a build name to it where the build's
    module tree differs from the reference's, e.g. the FLUX VAE decoder)."""
    rn = rename or (lambda n: n)
    return {f"base_model.model.{rn(n)}": p for n, p in model.named_parameters() if p.requires_grad}


def _save_adapter(model: torch.nn.Module, save_dir: Path, cfg_dict: Dict[str, Any],
                  rename: Optional[Callable[[str], str]] = None) -> None:
    from safetensors.torch import save_file
    save_dir = Path(save_dir)
    save_dir.mkdir(parents=True, exist_ok=True)
    tensors = {k: p.detach().float().cpu().contiguous() for k, p in _adapter_keys(model, rename).items()}
    save_file(tensors, str(save_dir / "adapter_model.safetensors"))
    (save_dir / "adapter_config.json").write_text(json.dumps(cfg_dict, indent=2))


def _load_adapter(model: torch.nn.Module, save_dir: Path, rename: Optional[Callable[[str], str]] = None) -> None:
    """Copy save_dir/adapter_model.safetensors back into the model's LoRA parameters.  Every trainable
    parameter must be present with its shape, and no extra key may exist (ValueError otherwise)."""
    from safetensors.torch import load_file
    tensors = load_file(str(Path(save_dir) / "adapter_model.safetensors"))
    want = _adapter_keys(model, rename)
    if set(tensors) != set(want):
        raise ValueError(f"adapter keys differ: missing {sorted(set(want) - set(tensors))[:3]}, "
                         f"unexpected {sorted(set(tensors) - set(want))[:3]}")
    with torch.no_grad():
        for k, p in want.items():
            if tuple(tensors[k].shape) != tuple(p.shape):
                raise ValueError(f"{k}: shape {tuple(tensors[k].shape)} != {tuple(p.shape)}")
            p.copy_(tensors[k].to(p.device, p.dtype))


def imagenet_prompt_text(class_id: int, labels_path: Union[str, Path] = "imagenet_classes.txt") -> str:
    """utills.py:216-273 without the download: "a photo of <label>" from a local labels file
    (one name per line); without one, the reference's own out-of-range fallback name class_<id>."""
    p = Path(labels_path)
    labels = [l.strip() for l in p.read_text(encoding="utf-8").splitlines() if l.strip()] if p.is_file() else []
    name = labels[class_id] if 0 <= class_id < len(labels) else f"class_{class_id}"
    return f"a photo of {name}"


@dataclass
class VarConfig:
    """es_backend.py:299-317 (+ build knobs).  Reference CLI defaults: unifed_es.py:396-406."""

    model_depth: int = 16
    ckpt_dir: str = "checkpoints_var"
    download_if_missing: bool = False
    guidance_scale: float = 4.0
    allowed_classes: Union[str, Sequence[int]] = "all"
    classes_per_gen: int = 2
    batches_per_gen: int = 4
    max_log_batches: int = 1
    torch_compile: bool = False
    compile_mode: str = "max-autotune"
    compile_fullgraph: bool = False
    lora_r: int = 4
    lora_alpha: int = 16
    lora_dropout: float = 0.0
    lora_target_modules: List[str] = field(default_factory=lambda: list(VAR_LORA_TARGETS))
    # build-specific
    arch: Optional[VARArch] = None          # None: VAR-d{model_depth} with the reference's VQVAE
    top_k: int = 900                        # models/VAR.py:276-277 generate() defaults
    top_p: float = 0.95
    labels_path: str = "imagenet_classes.txt"
    synthetic_if_missing: bool = False      # True: no checkpoint in ckpt_dir -> seeded synthetic weights (explicit opt-in)
    weight_seed: int = 0
    lora_seed: int = 1234
    lora_b_std: float = 0.02
    vae_chunk: int = 16


class VarBackend(ESBackend):
    """es_backend.py:319-450."""

    def __init__(self, device: str, cfg: VarConfig):
        self.name = "var_class"
        self.device = device
        self.cfg = cfg
        self.es_model: Optional[VARClassGenerator] = None
        self.image_pil_mode = 1          # rewards: the VAR PIL conversion (models/VAR.py:245-259)

    def init_and_attach_lora(self):
        c = self.cfg
        self.es_model = VARClassGenerator(model_depth=c.model_depth, device=self.device, arch=c.arch,
                                          weight_seed=c.weight_seed, vae_chunk=c.vae_chunk)
        d = Path(c.ckpt_dir)
        vae_ckpt, var_ckpt = d / "vae_ch160v4096z32.pth", d / f"var_d{self.es_model.model_depth}.pth"
        if vae_ckpt.is_file() and var_ckpt.is_file():
            self.es_model.load_reference_state(torch.load(var_ckpt, map_location="cpu", weights_only=True),
                                               torch.load(vae_ckpt, map_location="cpu", weights_only=True))
        elif not c.synthetic_if_missing:
            raise FileNotFoundError(f"Missing VAR checkpoints in {d} (no download offline)")
        n = attach_lora(self.es_model.transformer, c.lora_r, c.lora_alpha, c.lora_target_modules)
        if n == 0:
            raise RuntimeError("no LoRA target module matched")
        g = torch.Generator(device=self.device).manual_seed(c.lora_seed)
        for m in lora_modules(self.es_model.transformer):
            m.reset_lora(g, b_std=c.lora_b_std)
        self.es_model.transformer.eval()

    def collect_lora_params(self):
        return get_trainable_params_and_shapes(self.es_model.transformer)

    def save_lora(self, save_dir: Path) -> None:
        c = self.cfg
        _save_adapter(self.es_model.transformer, Path(save_dir),
                      {"peft_type": "LORA", "r": c.lora_r, "lora_alpha": c.lora_alpha, "lora_dropout": c.lora_dropout,
                       "target_modules": list(c.lora_target_modules),
                       "base_model_name_or_path": f"FoundationVision/var (depth={self.es_model.model_depth})",
                       "bias": "none", "task_type": None})

    def load_lora(self, save_dir: Path) -> None:
        """Inverse of save_lora (resume), see _load_adapter.  The mat_qkv LoRA entries round-trip too:
        they are in theta (perturbed, updated) even though the reference's F.linear bypasses them."""
        _load_adapter(self.es_model.transformer, Path(save_dir))

    def _sample_classes_unique(self, seed: int, num_classes_total: int = 1000) -> List[int]:
        return sample_classes_unique(seed, self.cfg.allowed_classes, self.cfg.classes_per_gen, num_classes_total)

    def step_sampling_info(self, seed: int) -> Dict[str, Any]:
        """es_backend.py:398-423."""
        unique_ids = self._sample_classes_unique(seed=seed, num_classes_total=1000)
        flat_ids = repeat_batches(unique_ids, repeats=self.cfg.batches_per_gen)
        m = len(unique_ids)
        txt = (lambda cid: imagenet_prompt_text(int(cid), self.cfg.labels_path))
        log_batches = int(max(0, min(self.cfg.max_log_batches, self.cfg.batches_per_gen)))
        return dict(unique_ids=unique_ids, flat_ids=flat_ids, unique_texts=[txt(c) for c in unique_ids],
                    flat_texts=[txt(c) for c in flat_ids], pid_to_j={cid: j for j, cid in enumerate(unique_ids)},
                    m=m, total_imgs_per_indiv=len(flat_ids), total_imgs_for_logging=log_batches * m,
                    log_batches=log_batches)

    def generate_flat(self, flat_ids: List[int], seed: int, guidance_scale: float,
                      flat_seeds: Optional[List[int]] = None) -> List[Any]:
        """es_backend.py:425-450: regroup flat_ids as [repeats][m], one generate call, flatten."""
        if flat_seeds is not None:
            raise NotImplementedError("VAR generation is seeded per call (g_seed), not per image")
        m, r = self.cfg.classes_per_gen, self.cfg.batches_per_gen
        if len(flat_ids) != m * r:
            raise RuntimeError(f"VAR expected flat_ids length {m*r}, got {len(flat_ids)}")
        grouped = [[int(flat_ids[b * m + j]) for j in range(m)] for b in range(r)]
        imgs, _ = self.es_model.generate(seed=seed, guidance_scale=guidance_scale, class_ids=grouped,
                                         return_grouped=True, top_k=self.cfg.top_k, top_p=self.cfg.top_p)
        return [imgs[b][j] for b in range(r) for j in range(m)]

    def generate_population(self, flat_ids: List[int], seed: int, guidance_scale: float,
                            theta_pop: torch.Tensor) -> torch.Tensor:
        """The grouped [repeats][m] class ids flatten back to flat_ids (models/VAR.py:206-242), so the
        label batch is flat_ids itself."""
        label = torch.as_tensor([int(c) for c in flat_ids], device=self.device, dtype=torch.long)
        return self.es_model.generate_population(label, theta_pop, seed, guidance_scale, self.cfg.top_k,
                                                 self.cfg.top_p)


# ---------------------------------------------------------------------------------------
# Z-Image-Turbo backend (es_backend.py:457-678) — BASELINE configs[3]
# ---------------------------------------------------------------------------------------


@dataclass
class ZImageConfig:
    """es_backend.py:457-495 (+ build knobs).  Reference CLI defaults: unifed_es.py:408-492."""

    model_name: str = "Tongyi-MAI/Z-Image-Turbo"
    prompts_txt_path: str = "untitled.txt"
    encoded_prompt_path: str = ""
    auto_encode_if_missing: bool = False
    width_px: int = 384
    height_px: int = 384
    num_inference_steps: int = 7
    guidance_scale: float = 0.0
    micro_batch: int = 1
    prompts_per_gen: int = 4
    batches_per_gen: int = 4
    max_log_batches: int = 1
    compile_transformer: bool = False
    attention_backend: str = "flash"
    use_gguf: bool = False
    lora_r: int = 2
    lora_alpha: int = 8
    lora_dropout: float = 0.0
    lora_target_modules: List[str] = field(default_factory=lambda: ["to_q", "to_k", "to_v", "linear", "w1", "w2", "w3"])
    use_vae_decoder_lora: bool = False
    vae_lora_r: int = 2                      # unifed_es.py:488-492 defaults
    vae_lora_alpha: int = 8
    vae_lora_dropout: float = 0.0
    vae_lora_target_modules: List[str] = field(default_factory=lambda: ["to_q", "to_k", "to_v", "to_out.0"])
    dtype: str = "bfloat16"
    # build-specific
    arch: Any = None                         # None: the Z-Image-Turbo config (zimage.ZIMAGE_TURBO)
    vae_widths: Tuple[int, ...] = (128, 256, 512, 512)
    vae_chunk: int = 16
    synthetic_prompts: int = 4               # used when encoded_prompt_path is empty
    synthetic_prompt_lens: Tuple[int, int] = (16, 100)
    lora_b_std: float = 0.02
    lora_seed: int = 1234
    weight_seed: int = 0
    synthetic_weights: bool = False          # no Z-Image checkpoint loader: True is required (explicit opt-in)


def synthetic_zimage_prompt_data(P: int = 4, lens: Tuple[int, int] = (16, 100), dim: int = 2560,
                                 seed: int = 0) -> Dict[str, Any]:
    """Same dict format as ZImageTurboES.encode_prompts (models/zImageTurbo.py:246-296): prompts and
    prompt_embeds = a list of per-prompt [T_i, dim] bf16 tensors (T_i ~ U[lens])."""
    g = torch.Generator().manual_seed(seed)
    T = torch.randint(lens[0], lens[1] + 1, (P,), generator=g).tolist()
    emb = [torch.randn(t, dim, generator=g).to(torch.bfloat16) for t in T]
    return {"prompts": [f"synthetic prompt {i}: a detailed photo of object {i}" for i in range(P)], "prompt_embeds": emb}


class ZImageBackend(ESBackend):
    """es_backend.py:498-678."""

    def __init__(self, device: str, cfg: ZImageConfig):
        self.name = "zimage"
        self.device = device
        self.cfg = cfg
        self.es_model = None
        self.prompt_data = None
        self.base_prompt_embeds = None
        self.prompts_list = None
        self.image_pil_mode = 0

    def _load_or_encode_prompts(self):
        """es_backend.py:515-562 (no text encoder offline: an encoded file or the synthetic set)."""
        if self.cfg.encoded_prompt_path:
            enc = Path(self.cfg.encoded_prompt_path)
            if not enc.is_file():
                raise FileNotFoundError(f"encoded_prompt_path not found and auto_encode unsupported: {enc}")
            self.prompt_data = torch.load(enc, map_location="cpu", weights_only=True)
        else:
            a = self.es_model.arch if self.es_model is not None else self.cfg.arch
            self.prompt_data = synthetic_zimage_prompt_data(self.cfg.synthetic_prompts, self.cfg.synthetic_prompt_lens,
                                                            a.cap_feat_dim if a is not None else 2560)
        self.base_prompt_embeds = self.prompt_data["prompt_embeds"]
        self.prompts_list = self.prompt_data.get("prompts", None)
        self._dev_prompts = [self._get_prompt_embed(p) for p in range(self._total_prompts())]

    def init_and_attach_lora(self):
        from .zimage import ZIMAGE_TURBO
        from .zimage_pipeline import ZImageTurboES
        from .lora import bind_theta_layout
        c = self.cfg
        self.es_model = ZImageTurboES(c.model_name, device=self.device, num_inference_steps=c.num_inference_steps,
                                      arch=c.arch or ZIMAGE_TURBO, vae_widths=c.vae_widths, vae_chunk=c.vae_chunk,
                                      weight_seed=c.weight_seed, synthetic_weights=c.synthetic_weights)
        self._load_or_encode_prompts()
        n = attach_lora(self.es_model.transformer, c.lora_r, c.lora_alpha, c.lora_target_modules)
        if n == 0:
            raise RuntimeError("no LoRA target module matched")
        g = torch.Generator(device=self.device).manual_seed(c.lora_seed)
        for m in lora_modules(self.es_model.transformer):
            m.reset_lora(g, b_std=c.lora_b_std)
        self.es_model.transformer.eval()
        if c.use_vae_decoder_lora:
            # es_backend.py:598-608: PEFT on the VAE decoder's mid-block attention linears; theta = the
            # transformer's trainable params then the decoder's (collect_lora_params, es_backend.py:613-618)
            vae = self.es_model.vae
            if attach_lora(vae, c.vae_lora_r, c.vae_lora_alpha, c.vae_lora_target_modules) == 0:
                raise RuntimeError("no VAE-decoder LoRA target module matched")
            d_tr = sum(p.numel() for p in self.es_model.transformer.parameters() if p.requires_grad)
            bind_theta_layout(vae, base=d_tr)
            for m in lora_modules(vae):
                m.reset_lora(g, b_std=c.lora_b_std)

    def collect_lora_params(self):
        tr_params, tr_shapes = get_trainable_params_and_shapes(self.es_model.transformer)
        if not self.cfg.use_vae_decoder_lora:
            return tr_params, tr_shapes
        vae_params, vae_shapes = get_trainable_params_and_shapes(self.es_model.vae)
        return tr_params + vae_params, tr_shapes + vae_shapes

    def _adapter_cfg(self, r, alpha, dropout, targets):
        return {"peft_type": "LORA", "r": r, "lora_alpha": alpha, "lora_dropout": dropout,
                "target_modules": list(targets), "base_model_name_or_path": self.cfg.model_name, "bias": "none",
                "task_type": None}

    def save_lora(self, save_dir: Path) -> None:
        """es_backend.py:611-619: the transformer adapter under save_dir/transformer (+ vae_decoder/)."""
        c = self.cfg
        _save_adapter(self.es_model.transformer, Path(save_dir) / "transformer",
                      self._adapter_cfg(c.lora_r, c.lora_alpha, c.lora_dropout, c.lora_target_modules))
        if c.use_vae_decoder_lora:
            # PEFT wraps pipe.vae.decoder (es_backend.py:598-608): keys carry diffusers' Decoder names
            # (base_model.model.mid_block.attentions.0.to_q.lora_A.weight), not flux_vae.py's (mid.1...)
            from .checkpoints import flux_decoder_name
            _save_adapter(self.es_model.vae, Path(save_dir) / "vae_decoder",
                          self._adapter_cfg(c.vae_lora_r, c.vae_lora_alpha, c.vae_lora_dropout,
                                            c.vae_lora_target_modules), rename=flux_decoder_name)

    def load_lora(self, save_dir: Path) -> None:
        _load_adapter(self.es_model.transformer, Path(save_dir) / "transformer")
        if self.cfg.use_vae_decoder_lora:
            from .checkpoints import flux_decoder_name
            _load_adapter(self.es_model.vae, Path(save_dir) / "vae_decoder", rename=flux_decoder_name)

    def _total_prompts(self) -> int:
        pe = self.base_prompt_embeds
        return len(pe) if isinstance(pe, list) else int(pe.shape[0])

    def _get_prompt_embed(self, pid: int) -> torch.Tensor:
        return self.base_prompt_embeds[pid].to(self.device)

    def step_sampling_info(self, seed: int) -> Dict[str, Any]:
        """es_backend.py:629-656."""
        unique_ids = sample_indices_unique(seed=seed, total=self._total_prompts(), k=self.cfg.prompts_per_gen)
        flat_ids = repeat_batches(unique_ids, repeats=self.cfg.batches_per_gen)
        m = len(unique_ids)
        name = (lambda pid: self.prompts_list[pid] if self.prompts_list is not None else f"prompt_{pid}")
        log_batches = int(max(0, min(self.cfg.max_log_batches, self.cfg.batches_per_gen)))
        return dict(unique_ids=unique_ids, flat_ids=flat_ids, unique_texts=[name(p) for p in unique_ids],
                    flat_texts=[name(p) for p in flat_ids], pid_to_j={pid: j for j, pid in enumerate(unique_ids)},
                    m=m, total_imgs_per_indiv=len(flat_ids), total_imgs_for_logging=log_batches * m,
                    log_batches=log_batches)

    def generate_flat(self, flat_ids: List[int], seed: int, guidance_scale: float,
                      flat_seeds: Optional[List[int]] = None) -> List[Any]:
        """es_backend.py:658-669: one member (the transformer's own LoRA params), PIL images."""
        if flat_seeds is not None:
            raise NotImplementedError("Z-Image latents are seeded per image from `seed` (per-prompt generators)")
        c = self.cfg
        images, _ = self.es_model.generate_one_batch([self._dev_prompts[p] for p in flat_ids], seed=seed,
                                                     guidance_scale=guidance_scale, width_px=c.width_px,
                                                     height_px=c.height_px, num_inference_steps=c.num_inference_steps,
                                                     micro_batch=c.micro_batch)
        return images

    def generate_population(self, flat_ids: List[int], seed: int, guidance_scale: float,
                            theta_pop: torch.Tensor) -> torch.Tensor:
        """The distinct prompts run the caption path once per member; image j keeps the latent of the
        reference's j-th per-prompt generator (seed + j)."""
        uniq = list(dict.fromkeys(int(f) for f in flat_ids))
        idx = torch.tensor([uniq.index(int(f)) for f in flat_ids], device=self.device)
        c = self.cfg
        return self.es_model.generate_population([self._dev_prompts[p] for p in uniq], idx, theta_pop, seed,
                                                 guidance_scale, c.width_px, c.height_px, c.num_inference_steps)


# ---------------------------------------------------------------------------------------
# Infinity (BASELINE configs[4]): es_backend.py:680-1023
# ---------------------------------------------------------------------------------------
@dataclass
class InfinityConfig:
    """es_backend.py:680-733; defaults = the reference CLI's 8b_512 variant (unifed_es.py:51-61, 422-472,
    micro_batch from --max_batch 2) + build knobs."""

    model_path: str = "Infinity/weights/infinity_8b_512x512_weights"
    text_encoder_ckpt: str = "google/flan-t5-xl"
    vae_path: str = "Infinity/weights/infinity_vae_d56_f8_14_patchify.pth"
    pn: str = "0.25M"
    model_type: str = "infinity_8b"
    vae_type: int = 14
    h_div_w_template: float = 1.0
    text_channels: int = 2048
    apply_spatial_patchify: int = 1
    use_flex_attn: int = 0
    bf16: int = 1
    checkpoint_type: str = "torch_shard"
    prompts_txt_path: str = "untitled1.txt"
    encoded_prompt_path: str = ""
    auto_encode_if_missing: bool = False
    encode_batch_size: int = 16
    drop_text_encoder_after_encode: bool = True
    prompts_per_gen: int = 4
    batches_per_gen: int = 4
    max_log_batches: int = 1
    cfg_list: Any = 3.0
    tau_list: Any = 1.0
    cfg_insertion_layer: int = 0
    sampling_per_bits: int = 1
    enable_positive_prompt: int = 0
    top_k: int = 900
    top_p: float = 0.97
    micro_batch: int = 2
    lora_r: int = 2
    lora_alpha: int = 8
    lora_dropout: float = 0.0
    lora_target_modules: List[str] = field(default_factory=lambda: ["fc1"])
    torch_compile: bool = False
    compile_mode: str = "max-autotune"
    compile_fullgraph: bool = False
    compile_vae: bool = False
    guidance_scale: float = 3.0              # --inf_guidance_scale (cfg_sc; the per-scale cfg_list applies)
    # build-specific
    arch: Any = None                         # None: arch_for(model_type, vae_type, apply_spatial_patchify)
    vae_chunk: int = 16
    kv_budget_gb: float = 120.0
    synthetic_prompts: int = 4               # used when encoded_prompt_path is empty
    synthetic_prompt_lens: Tuple[int, int] = (16, 100)
    lora_b_std: float = 0.02
    lora_seed: int = 1234
    weight_seed: int = 0
    synthetic_weights: bool = False          # no Infinity checkpoint loader: True is required (explicit opt-in)


def synthetic_infinity_prompt_data(P: int = 4, lens: Tuple[int, int] = (16, 100), dim: int = 2048,
                                   seed: int = 0) -> Dict[str, Any]:
    """Same dict format as InfinityES.encode_prompts (models/Infinity.py:267-335): prompts,
    kv_compact_list (per-prompt [L_i, dim] fp16 CPU tensors, L_i ~ U[lens]) and lens_list."""
    g = torch.Generator().manual_seed(seed)
    T = torch.randint(lens[0], lens[1] + 1, (P,), generator=g).tolist()
    kv = [(torch.randn(t, dim, generator=g) * 0.2).to(torch.float16) for t in T]
    return {"prompts": [f"synthetic prompt {i}: a detailed photo of object {i}" for i in range(P)],
            "kv_compact_list": kv, "lens_list": [int(t) for t in T]}


class InfinityBackend(ESBackend):
    """es_backend.py:735-1023."""

    def __init__(self, device: str, cfg: InfinityConfig):
        self.name = "infinity"
        self.device = device
        self.cfg = cfg
        self.es_model = None
        self.prompt_data = None
        self.kv_compact_list = None
        self.lens_list = None
        self.prompts_list = None
        self.image_pil_mode = 2          # rewards: Infinity's bf16 (x + 1) / 2 * 255 -> uint8

    def _load_or_encode_prompts(self):
        """es_backend.py:749-801 (no T5 offline: an encoded file, or the synthetic set when no path is set)."""
        c = self.cfg
        if c.encoded_prompt_path:
            enc = Path(c.encoded_prompt_path)
            if not enc.is_file():
                if not c.auto_encode_if_missing:
                    raise FileNotFoundError(f"encoded_prompt_path not found and auto_encode disabled: {enc}")
                raise FileNotFoundError(f"encoded_prompt_path not found and the T5 encoder is not available "
                                        f"offline: {enc}")
            self.prompt_data = torch.load(enc, map_location="cpu", weights_only=True)
        else:
            a = c.arch
            self.prompt_data = synthetic_infinity_prompt_data(c.synthetic_prompts, c.synthetic_prompt_lens,
                                                              a.text_channels if a is not None else c.text_channels)
        self.prompts_list = self.prompt_data["prompts"]
        self.kv_compact_list = self.prompt_data["kv_compact_list"]
        self.lens_list = self.prompt_data["lens_list"]
        self._dev_kv = [kv.to(self.device) for kv in self.kv_compact_list]

    def init_and_attach_lora(self) -> None:
        from .infinity_pipeline import InfinityES
        c = self.cfg
        self._load_or_encode_prompts()
        self.es_model = InfinityES(model_path=c.model_path, text_encoder_ckpt=c.text_encoder_ckpt, vae_path=c.vae_path,
                                   vae_type=int(c.vae_type), pn=c.pn, model_type=c.model_type,
                                   h_div_w_template=float(c.h_div_w_template), text_channels=int(c.text_channels),
                                   apply_spatial_patchify=int(c.apply_spatial_patchify),
                                   use_flex_attn=int(c.use_flex_attn), bf16=bool(c.bf16),
                                   checkpoint_type=c.checkpoint_type,
                                   enable_positive_prompt=int(c.enable_positive_prompt), top_k=int(c.top_k),
                                   top_p=float(c.top_p), cfg_insertion_layer=int(c.cfg_insertion_layer),
                                   sampling_per_bits=int(c.sampling_per_bits), device=self.device,
                                   synthetic_weights=c.synthetic_weights, arch=c.arch, weight_seed=c.weight_seed,
                                   vae_chunk=c.vae_chunk, kv_budget_gb=c.kv_budget_gb)
        n = attach_lora(self.es_model.transformer, c.lora_r, c.lora_alpha, c.lora_target_modules)
        if n == 0:
            raise RuntimeError("no LoRA target module matched")
        g = torch.Generator(device=self.device).manual_seed(c.lora_seed)
        for m in lora_modules(self.es_model.transformer):
            m.reset_lora(g, b_std=c.lora_b_std)
        self.es_model.infinity = self.es_model.transformer
        self.es_model.transformer.eval()
        self.es_model.drop_text_encoder()

    def compile_if_requested(self) -> None:
        return   # no tracing compiler on this stack: the hot ops are explicit libeggroll kernels

    def collect_lora_params(self):
        return get_trainable_params_and_shapes(self.es_model.transformer)

    def save_lora(self, save_dir: Path) -> None:
        """es_backend.py:820-822: the PEFT adapter of the transformer in save_dir."""
        c = self.cfg
        _save_adapter(self.es_model.transformer, Path(save_dir),
                      {"peft_type": "LORA", "r": c.lora_r, "lora_alpha": c.lora_alpha, "lora_dropout": c.lora_dropout,
                       "target_modules": list(c.lora_target_modules), "base_model_name_or_path": c.model_path,
                       "bias": "none", "task_type": None})

    def load_lora(self, save_dir: Path) -> None:
        _load_adapter(self.es_model.transformer, Path(save_dir))

    def step_sampling_info(self, seed: int) -> Dict[str, Any]:
        """es_backend.py:824-852."""
        P = int(len(self.kv_compact_list))
        unique_ids = sample_indices_unique(seed=seed, total=P, k=int(self.cfg.prompts_per_gen))
        flat_ids = repeat_batches(unique_ids, repeats=int(self.cfg.batches_per_gen))
        m = len(unique_ids)
        log_batches = int(max(0, min(int(self.cfg.max_log_batches), int(self.cfg.batches_per_gen))))
        return dict(unique_ids=unique_ids, flat_ids=flat_ids,
                    unique_texts=[self.prompts_list[p] for p in unique_ids],
                    flat_texts=[self.prompts_list[p] for p in flat_ids], pid_to_j={p: j for j, p in enumerate(unique_ids)},
                    m=m, total_imgs_per_indiv=len(flat_ids), total_imgs_for_logging=log_batches * m,
                    log_batches=log_batches)

    def generate_flat(self, flat_ids: List[int], seed: int, guidance_scale: float) -> List[Any]:
        """es_backend.py:893-1022: one member (the transformer's own LoRA params); micro_batch <= 0 or
        >= N is one call, else chunks of micro_batch images, each call reseeded with `seed`."""
        c = self.cfg
        if len(flat_ids) == 0:
            return []
        return self.es_model.generate_one_batch_from_compacts(
            kv_compact_list=[self._dev_kv[p] for p in flat_ids], lens_list=[int(self.lens_list[p]) for p in flat_ids],
            seed=seed, guidance_scale=guidance_scale, cfg_list=c.cfg_list, tau_list=c.tau_list,
            cfg_insertion_layer=int(c.cfg_insertion_layer), sampling_per_bits=int(c.sampling_per_bits),
            vae_type=int(c.vae_type), top_k=int(c.top_k), top_p=float(c.top_p), micro_batch=int(c.micro_batch))

    def generate_population(self, flat_ids: List[int], seed: int, guidance_scale: float,
                            theta_pop: torch.Tensor) -> torch.Tensor:
        """Every member's images in one batch per scale; the text path runs once per distinct prompt."""
        c = self.cfg
        uniq = list(dict.fromkeys(int(f) for f in flat_ids))
        idx = torch.tensor([uniq.index(int(f)) for f in flat_ids], device=self.device)
        return self.es_model.generate_population([self._dev_kv[p] for p in uniq], [int(self.lens_list[p]) for p in uniq],
                                                 idx, theta_pop, seed, c.cfg_list, c.tau_list, int(c.top_k),
                                                 float(c.top_p), int(c.micro_batch))
