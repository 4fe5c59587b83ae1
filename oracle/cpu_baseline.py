"""CPU baseline: the reference's ES hot path restated in numpy fp32 and timed on host cores.

TEST/BENCH INFRASTRUCTURE ONLY (imported by bench.py's cpu_baseline leg).  Follows the
reference's structure, not ours: members evaluated SEQUENTIALLY, eps [pop, D] MATERIALISED
(utills.py:70-106), per-member theta_k = theta + sigma*eps[k] + unflatten (unifed_es.py:160-161),
promptnorm + z-score (utills.py:168-178, 310-330), update (utills.py:115-136) and caps
(utills.py:333-349); and, per member, every PEFT-LoRA'd linear of the Sana transformer at its
real shape (y = x W^T + b + s (x A^T) B^T, fp32 like models/SanaSprint.py:35-39) with the
activation rows subsampled by `row_subsample` and the time scaled back linearly.
The non-LoRA parts of a member-eval (attention, FFN, VAE, reward networks) are NOT timed, so the
reported CPU member-evals/s is an UPPER bound on the CPU's full member-eval rate.
"""
from __future__ import annotations

import os
import time
from typing import Dict, List, Sequence, Tuple

import numpy as np

F32 = np.float32


def sana_lora_layers(images: int = 16, tokens: int = 1024, text_tokens: int = 300, blocks: int = 20
                     ) -> List[Tuple[int, int, int, int]]:
    """(rows_per_member, K, N, count) of the 168 LoRA targets of Sana-Sprint 1.6B."""
    D = 2240
    return [
        (images, 256, D, 2), (images, D, D, 2), (images, D, 6 * D, 1),           # time_embed (t, g, linear)
        (images * text_tokens, 2304, D, 1), (images * text_tokens, D, D, 1),    # caption_projection
        (images * tokens, D, D, 4 * blocks),                                      # attn1 q,k,v,out
        (images * tokens, D, D, 2 * blocks),                                      # attn2 q,out
        (images * text_tokens, D, D, 2 * blocks),                                 # attn2 k,v
        (images * tokens, D, 32, 1),                                              # proj_out
    ]


def lora_shapes_from_layers(layers, r: int = 2) -> List[Tuple[int, int]]:
    shapes = []
    for _, K, N, cnt in layers:
        for _ in range(cnt):
            shapes += [(r, K), (N, r)]
    return shapes


def es_arithmetic_epoch(shapes, pop: int, rank: int = 1, sigma: float = 1e-2, lr_scale: float = 1e-1,
                        theta_max_norm: float = 40.0, seed: int = 0) -> Dict[str, float]:
    rng = np.random.default_rng(seed)
    D = sum(int(np.prod(s)) for s in shapes)
    theta = (rng.standard_normal(D, dtype=F32) * F32(0.01))
    params = [np.empty(s, F32) for s in shapes]
    t0 = time.perf_counter()
    half, base = pop // 2, pop // 2 + pop % 2
    chunks = []
    for s in shapes:                                           # _sample_low_rank_block
        A = rng.standard_normal((base, s[0], rank), dtype=F32)
        B = rng.standard_normal((base, s[1], rank), dtype=F32)
        chunks.append((A @ B.transpose(0, 2, 1)).reshape(base, -1) / F32(np.sqrt(rank)))
    pos = np.concatenate(chunks, axis=1)
    eps = np.concatenate([pos[:half], -pos[:half]] + ([pos[half:half + 1]] if pop % 2 else []), axis=0)
    t1 = time.perf_counter()
    for k in range(pop):                                       # perturb + unflatten, per member
        th = theta + F32(sigma) * eps[k]
        idx = 0
        for p in params:
            p[...] = th[idx: idx + p.size].reshape(p.shape)
            idx += p.size
    t2 = time.perf_counter()
    S = rng.standard_normal((pop, 4), dtype=F32) + F32(21)
    mu = S.mean(0)
    c = S - mu
    sc = (c / max(np.sqrt((c * c).mean()), F32(1e-8))).mean(1)
    f = (sc - sc.mean()) / (sc.std(ddof=1) + F32(1e-8))
    t3 = time.perf_counter()
    g = (f[:, None] * eps).mean(0)
    new = theta + F32(lr_scale * sigma) * g
    n = np.linalg.norm(new)
    if n > theta_max_norm:
        new = new * F32(theta_max_norm / (n + 1e-8))
    t4 = time.perf_counter()
    return {"sample_eps_s": t1 - t0, "perturb_s": t2 - t1, "fitness_s": t3 - t2, "update_s": t4 - t3,
            "total_s": t4 - t0, "D": D}


def lora_stack_member(layers, r: int = 2, row_subsample: int = 64, seed: int = 0) -> Dict[str, float]:
    """One member's perturbed LoRA linears (distinct weights per shape class; same FLOPs)."""
    rng = np.random.default_rng(seed)
    cache = {}
    total = 0.0
    flops = 0.0
    for rows, K, N, cnt in layers:
        key = (K, N)
        if key not in cache:
            cache[key] = (rng.standard_normal((N, K), dtype=F32) * F32(0.02), rng.standard_normal(N, dtype=F32),
                          rng.standard_normal((r, K), dtype=F32) * F32(0.02),
                          rng.standard_normal((N, r), dtype=F32) * F32(0.02))
        W, b, A, B = cache[key]
        m = max(1, rows // row_subsample)
        x = rng.standard_normal((m, K), dtype=F32)
        t0 = time.perf_counter()
        for _ in range(cnt):
            y = x @ W.T + b + F32(4.0) * ((x @ A.T) @ B.T)
        total += (time.perf_counter() - t0) * (rows / m)
        flops += cnt * 2.0 * rows * K * N
    return {"lora_stack_s": total, "lora_flops": flops}


def run(pop: int = 8, rank: int = 1, r: int = 2, row_subsample: int = 64, budget_s: float = 15.0) -> Dict[str, object]:
    cores = int(os.environ.get("OMP_NUM_THREADS", "0")) or len(os.sched_getaffinity(0))
    layers = sana_lora_layers()
    shapes = lora_shapes_from_layers(layers, r)
    t_start = time.perf_counter()
    es = es_arithmetic_epoch(shapes, pop, rank)
    reps, stack = 0, 0.0
    while True:
        stack += lora_stack_member(layers, r, row_subsample, seed=reps)["lora_stack_s"]
        reps += 1
        if time.perf_counter() - t_start > budget_s or reps >= 4:
            break
    per_member = stack / reps + es["total_s"] / pop
    try:
        cpu = next((ln.split(":", 1)[1].strip() for ln in open("/proc/cpuinfo") if ln.startswith("model name")), "?")
    except OSError:
        cpu = "?"
    return {"value": 1.0 / per_member, "unit": "member-evals/s", "cores": cores, "kind": "port",
            "sample": (f"numpy fp32 restatement of the reference path, pop={pop} (D={es['D']}): ES arithmetic per epoch "
                       f"({es['total_s']:.2f}s: materialised eps, sequential perturb+unflatten, promptnorm, update, cap) "
                       f"+ per-member LoRA-linear stack (168 Sana linears at 1024px, rows subsampled 1/{row_subsample}, "
                       f"time scaled x{row_subsample}, {reps} member(s) timed = {stack / reps:.2f}s/member); "
                       f"attention/FFN/VAE/reward networks not timed -> upper bound; cpu={cpu}"),
            "es_breakdown_s": {k: v for k, v in es.items() if k.endswith("_s")},
            "wall_s": time.perf_counter() - t_start}


if __name__ == "__main__":
    import json
    print(json.dumps(run(budget_s=5.0), indent=1))
