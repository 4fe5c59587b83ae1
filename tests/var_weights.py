"""Deterministic synthetic weights for the VAR model-level parity fixture (g11), test infrastructure.

The same recipe is applied to the reference's VAR / VQVAE modules when the fixture is generated
(tests/golden/make_golden.py, this container) and to this build's modules on the GPU box: both
module trees carry the reference's parameter names, so name -> tensor is all that must agree.
Every tensor comes from its own CPU generator seeded by (seed, its name), so the result does not
depend on iteration order or on the device the model lives on.
"""
from __future__ import annotations

import math
import zlib
from typing import Dict, Iterable, Tuple

import torch

TINY = dict(depth=2, vae_ch=32, lora_r=4, lora_alpha=16.0)
TARGETS = ["mat_qkv", "proj", "fc1", "fc2", "ada_lin.1", "head_nm.ada_lin.1", "head"]   # unifed_es.py:406


def synth_tensor(name: str, shape: Tuple[int, ...], seed: int) -> torch.Tensor:
    g = torch.Generator().manual_seed(seed * 1_000_003 + zlib.crc32(name.encode()))
    z = torch.randn(shape, generator=g, dtype=torch.float32)
    if name.endswith("quantize.embedding.weight"):
        return z
    if name.endswith(("class_emb.weight", "lvl_embed.weight", "pos_start", "pos_1LC")):
        return z * 0.3
    if name.endswith("scale_mul_1H11"):
        return math.log(4.0) + 0.1 * z
    if len(shape) == 1:
        if "norm" in name and name.endswith("weight"):
            return 1.0 + 0.1 * z
        return 0.05 * z
    fan_in = math.prod(shape[1:])
    mult = 0.5 if "ada_lin" in name else 1.0
    return z * (mult / math.sqrt(fan_in))


def synth_state(named_shapes: Iterable[Tuple[str, Tuple[int, ...]]], seed: int = 11) -> Dict[str, torch.Tensor]:
    return {n: synth_tensor(n, tuple(s), seed) for n, s in named_shapes}


def synth_theta(lora_shapes, seed: int = 12) -> torch.Tensor:
    """LoRA theta in the reference layout: lora_A ~ U(+-1/sqrt(in)) (PEFT kaiming bound), lora_B ~ N(0, 0.05)."""
    g = torch.Generator().manual_seed(seed)
    parts = []
    for i, (a, b) in enumerate(lora_shapes):
        if i % 2 == 0:   # lora_A [r, in]
            parts.append((torch.rand((a, b), generator=g) * 2 - 1).div_(math.sqrt(b)).reshape(-1))
        else:            # lora_B [out, r]
            parts.append(torch.randn((a, b), generator=g).mul_(0.05).reshape(-1))
    return torch.cat(parts)
