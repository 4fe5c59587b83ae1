"""CPU baseline: the reference's ES epoch restated in fp32 torch-CPU and timed on the host cores
(BASELINE.md §3 rows CPU-1 / CPU-2 / CPU-3).

TEST/BENCH INFRASTRUCTURE ONLY (imported by bench.py's cpu_baseline leg).  It follows the
reference's structure, not the build's: members evaluated SEQUENTIALLY, eps [pop, D] MATERIALISED
(utills.py:43-106), per-member theta_k = theta + sigma * eps[k] + unflatten into the LoRA params
(unifed_es.py:159-161), promptnorm + z-score (utills.py:168-178, 310-330), update (utills.py:115-136)
and cap (utills.py:333-339), all fp32 on `torch.set_num_threads(cores)`.

  CPU-1  ES arithmetic of one epoch at N = 64, Sana-Sprint 1.6B LoRA layout (D = 1,515,456, r_e 1).
  CPU-2  One member-eval, every op of it at its real width, through the fp32 restatement of the
         member path (oracle/member_eval_fp32.py, the same code the GPU parity test checks the build
         against): the Sana transformer at 1024 px with 2 of its 20 blocks (+ embeddings, caption
         projection, head) on 1 of the member's 16 images, the DC-AE decoder on 1 image at 1/16 of the
         1024^2 pixels (a 256 px crop: fully convolutional + linear attention, cost linear in pixels),
         and the CLIP-H/14 (4 of 32 vision layers) + CLIP-B/32 image towers on 1 image.  Each timed part
         is scaled linearly (blocks x10, images x16, pixels x16, layers x8); text towers run once per
         epoch and are left out.  All 100 % of the member-eval's op types are timed; the scaling
         factors are stated in the sample string.
  CPU-3  ES arithmetic of one epoch for the plumbing config: VAR-d16 layout (D = 1,540,096, LoRA r 4),
         N = 4.
value = 1 / (CPU-2 seconds per member + CPU-1 seconds / 64)  member-evals/s.
"""
from __future__ import annotations

import math
import os
import time
from typing import Dict, List, Sequence, Tuple

import torch

f32 = torch.float32


def cpu_threads() -> int:
    """Threads actually used: the affinity mask, capped by OMP_NUM_THREADS when set (the GPU box
    exports 16; os.sched_getaffinity there lists the whole machine)."""
    n = len(os.sched_getaffinity(0))
    omp = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
    return min(n, omp) if omp > 0 else n


# ----------------------------------------------------------------------------------------------
# CPU-1 / CPU-3: the reference's ES arithmetic (utills.py restated in torch, same op sequence)
# ----------------------------------------------------------------------------------------------


def _sample_eps(shapes: Sequence[Tuple[int, ...]], pop: int, rank: int, gen: torch.Generator) -> torch.Tensor:
    """EggRollNoiser.sample_eps (utills.py:43-106), antithetic."""
    half = pop // 2
    base = half + pop % 2
    chunks = []
    for s in shapes:
        if len(s) == 2:
            A = torch.randn(base, s[0], rank, generator=gen)
            B = torch.randn(base, s[1], rank, generator=gen)
            chunks.append((A @ B.transpose(1, 2)).reshape(base, -1) / math.sqrt(rank))
        else:
            chunks.append(torch.randn(base, int(math.prod(s)), generator=gen))
    pos = torch.cat(chunks, dim=1)
    parts = [pos[:half], -pos[:half]] + ([pos[half:half + 1]] if pop % 2 else [])
    return torch.cat(parts, dim=0)


def es_arithmetic_epoch(shapes, pop: int, rank: int = 1, sigma: float = 1e-2, lr_scale: float = 1e-1,
                        theta_max_norm: float = 40.0, seed: int = 0) -> Dict[str, float]:
    gen = torch.Generator().manual_seed(seed)
    D = sum(int(math.prod(s)) for s in shapes)
    theta = torch.randn(D, generator=gen) * 0.01
    params = [torch.empty(s) for s in shapes]
    t0 = time.perf_counter()
    eps = _sample_eps(shapes, pop, rank, gen)
    t1 = time.perf_counter()
    for k in range(pop):                                       # unifed_es.py:159-161
        th = theta + sigma * eps[k]
        idx = 0
        for p in params:
            p.copy_(th[idx: idx + p.numel()].view(p.shape))
            idx += p.numel()
    t2 = time.perf_counter()
    S = torch.randn(pop, 4, generator=gen) + 21               # utills.py:310-330 then 168-178
    mu = S.mean(dim=0)
    C = S - mu
    sb = torch.sqrt((C * C).mean()).clamp_min(1e-8)
    scores = (C / sb).mean(dim=1)
    std = scores.std()
    f = torch.zeros_like(scores) if std < 1e-8 else (scores - scores.mean()) / (std + 1e-8)
    t3 = time.perf_counter()
    new = theta + (lr_scale * sigma) * (f.unsqueeze(1) * eps).mean(dim=0)   # utills.py:115-136
    n = new.norm()
    if n > theta_max_norm:                                      # utills.py:333-339
        new = new * (theta_max_norm / (n + 1e-8))
    t4 = time.perf_counter()
    return {"sample_eps_s": t1 - t0, "perturb_unflatten_s": t2 - t1, "fitness_s": t3 - t2, "update_cap_s": t4 - t3,
            "total_s": t4 - t0, "D": D, "pop": pop}


# ----------------------------------------------------------------------------------------------
# CPU-2: one member-eval through the fp32 restatement, sub-sampled and scaled
# ----------------------------------------------------------------------------------------------


def member_eval(seed: int = 0) -> Dict[str, float]:
    from hyperscalees_t2i_amd.dcae import DCAEDecoder
    from hyperscalees_t2i_amd.lora import lora_modules
    from hyperscalees_t2i_amd.rewards import CLIP_B32, CLIP_H14, build_clip, clip_preprocess, postprocess_uint8
    from hyperscalees_t2i_amd.sana import SANA_LORA_TARGETS, SanaArch, SanaTransformer2DModel, attach_lora

    from . import member_eval_fp32 as R

    full = SanaArch()
    blocks_timed = 2
    arch = SanaArch(num_layers=blocks_timed)
    tr = SanaTransformer2DModel(arch)
    tr.init_weights(seed)
    attach_lora(tr, 2, 8.0, SANA_LORA_TARGETS)
    g = torch.Generator().manual_seed(seed + 1)
    for m in lora_modules(tr):
        m.reset_lora(g, b_std=0.02)
    theta_k = torch.cat([p.detach().reshape(-1) for p in tr.parameters() if p.requires_grad]).float()
    vae = DCAEDecoder(arch.in_channels)
    vae.init_weights(seed + 2)
    ccfg = {k: dict(v) if isinstance(v, dict) else v for k, v in CLIP_H14.items()}
    vis_layers = ccfg["vision_config"]["num_hidden_layers"]
    ccfg["vision_config"]["num_hidden_layers"] = 4
    ccfg["text_config"]["num_hidden_layers"] = 1
    clip_h = build_clip(ccfg, "cpu", seed + 3, dtype=f32)
    clip_b = build_clip(CLIP_B32, "cpu", seed + 4, dtype=f32)

    lat = torch.randn(1, 32, 32, 32, generator=g) * 0.5
    pe = torch.randn(1, 300, 2304, generator=g)
    am = torch.ones(1, 300, dtype=torch.int64)
    t = torch.full((1,), 0.5)
    gs = torch.full((1,), 0.45)
    out = {}
    with torch.no_grad():
        R.transformer_fp32(tr, theta_k, lat[:, :, :8, :8], t, pe[:, :16], am[:, :16], gs)   # warm-up
        t0 = time.perf_counter()
        R.transformer_fp32(tr, theta_k, lat, t, pe, am, gs)
        out["transformer_1img_2blk_s"] = time.perf_counter() - t0
        z = torch.randn(1, 32, 8, 8, generator=g)                                            # 256 px output
        R.dcae_fp32(vae, z[:, :, :2, :2])
        t0 = time.perf_counter()
        img = R.dcae_fp32(vae, z)
        out["dcae_1img_256px_s"] = time.perf_counter() - t0
        px = clip_preprocess(postprocess_uint8(img.clamp(-1, 1)))
        t0 = time.perf_counter()
        clip_h.visual_projection(clip_h.vision_model(pixel_values=px).pooler_output)
        out["clip_h_1img_4layers_s"] = time.perf_counter() - t0
        t0 = time.perf_counter()
        clip_b.visual_projection(clip_b.vision_model(pixel_values=px).pooler_output)
        out["clip_b_1img_s"] = time.perf_counter() - t0
    images = 16
    # transformer: the 2 timed blocks scale to 20; embeddings / caption / head are counted once per image
    # (they are < 3 % of one block's cost, so the linear block scaling is a slight over-estimate)
    per_img_tr = out["transformer_1img_2blk_s"] * full.num_layers / blocks_timed
    per_img_vae = out["dcae_1img_256px_s"] * 16.0
    per_img_rew = out["clip_h_1img_4layers_s"] * vis_layers / 4 + out["clip_b_1img_s"]
    out["member_eval_s"] = images * (per_img_tr + per_img_vae + per_img_rew)
    out["scale"] = (f"transformer {blocks_timed}/{full.num_layers} blocks x{full.num_layers // blocks_timed}, "
                    f"DC-AE 256px x16 pixels, CLIP-H {4}/{vis_layers} layers x{vis_layers // 4}, images x{images}")
    return out


def run(pop: int = 64, budget_s: float = 30.0) -> Dict[str, object]:
    from hyperscalees_t2i_amd.model_shapes import var_d16_lora_shapes
    from hyperscalees_t2i_amd.sana import sana_lora_shapes
    cores = cpu_threads()
    prev = torch.get_num_threads()
    torch.set_num_threads(cores)
    t_start = time.perf_counter()
    try:
        cpu1 = es_arithmetic_epoch(sana_lora_shapes(), 64, rank=1)
        cpu3 = es_arithmetic_epoch(var_d16_lora_shapes(), 4, rank=1)
        cpu2 = member_eval()
    finally:
        torch.set_num_threads(prev)
    per_member = cpu2["member_eval_s"] + cpu1["total_s"] / 64
    try:
        cpu = next((ln.split(":", 1)[1].strip() for ln in open("/proc/cpuinfo") if ln.startswith("model name")), "?")
    except OSError:
        cpu = "?"
    return {"value": 1.0 / per_member, "unit": "member-evals/s", "cores": cores, "kind": "port",
            "sample": (f"fp32 torch-CPU restatement of the reference path on {cores} threads ({cpu}). "
                       f"CPU-1: ES arithmetic, Sana layout D={cpu1['D']}, N=64: {cpu1['total_s']:.3f}s/epoch "
                       f"(sample_eps {cpu1['sample_eps_s']:.3f}, 64x perturb+unflatten {cpu1['perturb_unflatten_s']:.3f}, "
                       f"update+cap {cpu1['update_cap_s']:.3f}). "
                       f"CPU-2: one member-eval (16 images at 1024px: transformer + DC-AE + CLIP-H/CLIP-B) through "
                       f"oracle/member_eval_fp32.py, timed on a sub-sample and scaled linearly ({cpu2['scale']}): "
                       f"{cpu2['member_eval_s']:.1f}s/member. "
                       f"CPU-3: ES arithmetic, VAR-d16 layout D={cpu3['D']}, N=4: {cpu3['total_s']:.3f}s/epoch. "
                       f"value = 1/(CPU-2 + CPU-1/64)"),
            "rows": {"CPU-1": cpu1, "CPU-2": {k: v for k, v in cpu2.items()}, "CPU-3": cpu3},
            "wall_s": time.perf_counter() - t_start}


if __name__ == "__main__":
    import json
    print(json.dumps(run(), indent=1, default=str))
