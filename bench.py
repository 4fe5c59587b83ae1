#!/usr/bin/env python3
"""Benchmark: ES member-evals/sec (whole node) for the Sana-Sprint 1.6B one-step EGGROLL epoch.

    python bench.py [--gpus N] [--steps K] [--warmup W]
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
        --master-port P bench.py --gpus N --steps K --warmup W

One step = one full ES epoch (noise -> perturb -> population forward of the 1.6B transformer at
1024 px -> DC-AE decode -> CLIP-B/32 + PickScore rewards -> S all-gather -> promptnorm fitness ->
update) with pop_per_gpu = 8 members per GPU (weak scaling: N=1 is BASELINE configs[1], pop 8;
N=8 is configs[2], pop 64).  value = pop_total * K / max-over-ranks wall time of the K timed epochs.
Synthetic data: random-init frozen weights of the Sana/DC-AE/CLIP architectures (no checkpoints
offline), synthetic prompt embeddings, random-init LoRA.

Extra fields: `roofline` of the dominant hand-written kernel (the population LoRA GEMM, MFMA-bound,
timed live with HIP events on its launch stream during the timed epochs), `cpu_baseline` (the
reference path restated in numpy, timed on this host's cores; rank 0, N=1 only), per-phase times.
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys
import time
from pathlib import Path

os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
os.environ.setdefault("MIOPEN_DEBUG_CONV_DIRECT_NAIVE_CONV_FWD", "0")  # see hyperscalees_t2i_amd/__init__.py
ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT))

import torch  # noqa: E402

# MIOpen Find per conv shape during warmup (FAST mode: 38 vs 700+ TF); Find picks solvers by timing, so two
# processes can pick different ones for the same shape: EGGROLL_MIOPEN_FIND=0 (MIOpen's immediate mode)
# makes the choice a function of the shape only (tests/test_gpu_bench_dist.py compares processes bitwise)
torch.backends.cudnn.benchmark = os.environ.get("EGGROLL_MIOPEN_FIND", "1") == "1"
T_START = time.perf_counter()


def log(msg: str) -> None:
    print(f"[bench +{time.perf_counter() - T_START:7.1f}s] {msg}", file=sys.stderr, flush=True)


def start_heartbeat(period_s: float = 30.0) -> None:
    """Progress line every `period_s` on stderr (MIOpen Find during warmup can run for minutes
    without returning to Python; torch releases the GIL inside ops, so this thread keeps ticking)."""
    import threading

    def beat():
        while True:
            time.sleep(period_s)
            log("heartbeat")

    threading.Thread(target=beat, daemon=True).start()

METRIC = "ES member-evals/sec (whole node) Sana-Sprint 1.6B pop=64; % HBM/MFMA roofline"
BF16_DENSE_PEAK_TFLOPS = 2500.0   # MI355X_MICROARCH.md: ~2.5 PF dense bf16
HBM_PEAK_GBPS = 8000.0            # MI355X_MICROARCH.md: 8.0 TB/s spec


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=3)
    p.add_argument("--warmup", type=int, default=1)
    p.add_argument("--pop-per-gpu", type=int, default=8)
    p.add_argument("--latent", type=int, default=32, help="32 -> 1024 px")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--small", action="store_true", help="tiny architecture (smoke only; not a valid metric)")
    p.add_argument("--aux-out", type=str, default="",
                   help="write the full record (per-phase / per-kernel tables) here; default gpurun_out/bench_aux.json")
    p.add_argument("--workload", choices=("sana", "var_d16", "zimage", "infinity"), default="sana",
                   help="var_d16: BASELINE configs[0] (VAR-d16, LoRA r 4, 4 classes x 4 batches) on the GPU path; "
                        "zimage: configs[3] (Z-Image-Turbo, egg rank 4, one GPU's 16 of pop 128, 384 px, 7 steps); "
                        "infinity: configs[4] (Infinity-8B 512 px, one GPU's 4 of pop 32, 10 scales, cfg 3)")
    a = p.parse_args()
    if a.workload == "var_d16" and a.pop_per_gpu == 8 and "--pop-per-gpu" not in sys.argv:
        a.pop_per_gpu = 4           # configs[0]: pop_size 4
    if a.workload == "zimage" and a.pop_per_gpu == 8 and "--pop-per-gpu" not in sys.argv:
        a.pop_per_gpu = 16          # configs[3]: pop_size 128 across 8 GPUs
    if a.workload == "infinity" and a.pop_per_gpu == 8 and "--pop-per-gpu" not in sys.argv:
        a.pop_per_gpu = 4           # configs[4]: pop_size 32 across 8 GPUs
    return a


def dist_setup(args):
    """One process per GPU (torchrun env).  RCCL ("nccl") by default; EGGROLL_DIST_BACKEND=gloo with
    EGGROLL_SAME_DEVICE=1 rehearses the N>1 path with every rank on cuda:0 (a 1-GPU box)."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if os.environ.get("EGGROLL_SAME_DEVICE") == "1":
        local = 0
    torch.cuda.set_device(local)
    if world > 1:
        import torch.distributed as dist
        backend = os.environ.get("EGGROLL_DIST_BACKEND", "nccl")
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device(f"cuda:{local}"))
        else:
            dist.init_process_group(backend)
    return rank, world, local


def barrier(world):
    if world > 1:
        import torch.distributed as dist
        dist.barrier()


def max_over_ranks(x: float, world: int) -> float:
    if world == 1:
        return x
    import torch.distributed as dist
    t = torch.tensor([x], device="cuda", dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def build_var(args, world, rank, device):
    """BASELINE configs[0]: VAR-d16 class-conditional, LoRA r 4 / alpha 16 on the reference targets,
    pop 4 antithetic, 4 classes x 4 batches per member (16 images at 256 px), cfg 4, top-k 900 / top-p 0.95."""
    from hyperscalees_t2i_amd.backend import VarBackend, VarConfig
    from hyperscalees_t2i_amd.es import EggRollNoiser, flatten_params
    from hyperscalees_t2i_amd.es_step import DistInfo, ESConfig, ESEngine
    from hyperscalees_t2i_amd.rewards import RewardModels
    from hyperscalees_t2i_amd.var import VARArch

    cfg = VarConfig(classes_per_gen=4, batches_per_gen=4, synthetic_if_missing=True)
    if args.small:
        cfg.arch = VARArch(depth=2, vae_ch=32)
    backend = VarBackend(device=str(device), cfg=cfg)
    backend.init_and_attach_lora()
    params, shapes = backend.collect_lora_params()
    theta = flatten_params(params).to(device=device, dtype=torch.float32)
    noiser = EggRollNoiser(shapes, sigma=1e-2, lr_scale=1e-1, rank=1, use_antithetic=True)
    rewards = RewardModels.build(device, tiny=args.small, synthetic=True)
    pop = args.pop_per_gpu * world
    es_cfg = ESConfig(pop_size=pop, sigma=1e-2, lr_scale=1e-1, egg_rank=1, use_antithetic=True, promptnorm=True,
                      theta_max_norm=40.0, max_step_norm=0.0)
    engine = ESEngine(backend, rewards, noiser, es_cfg, device, DistInfo(rank, world, None))
    return backend, engine, noiser, theta, pop


def build_zimage(args, world, rank, device):
    """BASELINE configs[3]: Z-Image-Turbo LoRA ES, LoRA r 2 / alpha 8 on to_q,to_k,to_v,linear,w1,w2,w3,
    egg rank 4, pop_per_gpu (16 = one GPU's share of pop 128) antithetic, 4 prompts x 4 batches per member
    at 384 px, 7 flow-matching steps, guidance 0 (unifed_es.py:408-492 defaults)."""
    from hyperscalees_t2i_amd.backend import ZImageBackend, ZImageConfig
    from hyperscalees_t2i_amd.es import EggRollNoiser, flatten_params
    from hyperscalees_t2i_amd.es_step import DistInfo, ESConfig, ESEngine
    from hyperscalees_t2i_amd.rewards import RewardModels
    from hyperscalees_t2i_amd.zimage import ZImageArch

    cfg = ZImageConfig(synthetic_weights=True)
    if args.small:
        cfg.arch = ZImageArch(dim=256, n_layers=2, n_refiner_layers=1, n_heads=2, ffn=512, cap_feat_dim=256, t_mid=256,
                              seq_multiple=16)   # 64 px: 16 image tokens
        cfg.vae_widths, cfg.width_px, cfg.height_px, cfg.num_inference_steps = (32, 32, 64, 64), 64, 64, 2
    backend = ZImageBackend(device=str(device), cfg=cfg)
    backend.init_and_attach_lora()
    params, shapes = backend.collect_lora_params()
    theta = flatten_params(params).to(device=device, dtype=torch.float32)
    noiser = EggRollNoiser(shapes, sigma=1e-2, lr_scale=1e-1, rank=4, use_antithetic=True)
    rewards = RewardModels.build(device, tiny=args.small, synthetic=True)
    pop = args.pop_per_gpu * world
    es_cfg = ESConfig(pop_size=pop, sigma=1e-2, lr_scale=1e-1, egg_rank=4, use_antithetic=True, promptnorm=True,
                      theta_max_norm=40.0, max_step_norm=0.0)
    engine = ESEngine(backend, rewards, noiser, es_cfg, device, DistInfo(rank, world, None))
    return backend, engine, noiser, theta, pop


def build_infinity(args, world, rank, device):
    """BASELINE configs[4]: Infinity-8B 512 px (pn 0.25M, f8 VAE + 2x2 patchify, 14 bits per VAE pixel),
    LoRA r 2 / alpha 8 on fc1, egg rank 1, pop_per_gpu (4 = one GPU's share of pop 32) antithetic,
    4 prompts x 4 batches per member, cfg 3 / tau 1 / top-k 900 / top-p 0.97, micro_batch 2
    (unifed_es.py:51-61, 422-472 defaults)."""
    from hyperscalees_t2i_amd.backend import InfinityBackend, InfinityConfig
    from hyperscalees_t2i_amd.es import EggRollNoiser, flatten_params
    from hyperscalees_t2i_amd.es_step import DistInfo, ESConfig, ESEngine
    from hyperscalees_t2i_amd.infinity import InfinityArch
    from hyperscalees_t2i_amd.rewards import RewardModels

    cfg = InfinityConfig(synthetic_weights=True)
    if args.small:
        cfg.arch = InfinityArch(depth=2, embed_dim=256, num_heads=2, block_chunks=2, text_channels=256,
                                codebook_dim=4, spatial_patchify=1, vae_widths=(32, 32, 64, 64))
        cfg.pn = "0.06M"
    backend = InfinityBackend(device=str(device), cfg=cfg)
    backend.init_and_attach_lora()
    params, shapes = backend.collect_lora_params()
    theta = flatten_params(params).to(device=device, dtype=torch.float32)
    noiser = EggRollNoiser(shapes, sigma=1e-2, lr_scale=1e-1, rank=1, use_antithetic=True)
    rewards = RewardModels.build(device, tiny=args.small, synthetic=True)
    pop = args.pop_per_gpu * world
    es_cfg = ESConfig(pop_size=pop, sigma=1e-2, lr_scale=1e-1, egg_rank=1, use_antithetic=True, promptnorm=True,
                      theta_max_norm=40.0, max_step_norm=0.0)
    engine = ESEngine(backend, rewards, noiser, es_cfg, device, DistInfo(rank, world, None))
    return backend, engine, noiser, theta, pop


def build(args, world, rank, device):
    if args.workload == "infinity":
        return build_infinity(args, world, rank, device)
    if args.workload == "var_d16":
        return build_var(args, world, rank, device)
    if args.workload == "zimage":
        return build_zimage(args, world, rank, device)
    from hyperscalees_t2i_amd.backend import SanaBackend, SanaConfig
    from hyperscalees_t2i_amd.es import EggRollNoiser, flatten_params
    from hyperscalees_t2i_amd.es_step import DistInfo, ESConfig, ESEngine
    from hyperscalees_t2i_amd.rewards import RewardModels
    from hyperscalees_t2i_amd.sana import SanaArch

    cfg = SanaConfig(synthetic_weights=True, width_latent=args.latent, height_latent=args.latent)
    if args.small:
        # cross-attention head dim 112 as the full model, so attn2 runs eggroll_cross_attention (run-to-run
        # deterministic) rather than the SDPA fallback (masked SDPA at head dim 64 is not: tools/
        # sdpa_determinism_probe.py) — the multi-process tests compare theta' across processes bitwise
        cfg.arch = SanaArch(num_attention_heads=14, attention_head_dim=32, num_layers=2, num_cross_attention_heads=4,
                            cross_attention_head_dim=112, caption_channels=256)   # inner 448: K % 64 == 0
        cfg.vae_widths, cfg.vae_layers = (16, 32, 32, 64, 64, 64), (1, 1, 1, 1, 1, 1)
    backend = SanaBackend(device=str(device), cfg=cfg)
    backend.init_and_attach_lora()
    if args.small:  # synthetic prompt embeds must match the tiny caption width
        backend.base_prompt_embeds = backend.base_prompt_embeds[..., :256].contiguous()
        backend._dev_prompts = (backend.base_prompt_embeds.to(device), backend.base_attention_mask.to(device))
    params, shapes = backend.collect_lora_params()
    theta = flatten_params(params).to(device=device, dtype=torch.float32)
    noiser = EggRollNoiser(shapes, sigma=1e-2, lr_scale=1e-1, rank=1, use_antithetic=True)
    rewards = RewardModels.build(device, tiny=args.small, synthetic=True)
    pop = args.pop_per_gpu * world
    es_cfg = ESConfig(pop_size=pop, sigma=1e-2, lr_scale=1e-1, egg_rank=1, use_antithetic=True, promptnorm=True,
                      theta_max_norm=40.0, max_step_norm=0.0)
    engine = ESEngine(backend, rewards, noiser, es_cfg, device, DistInfo(rank, world, None))
    return backend, engine, noiser, theta, pop


def marker():
    """One tiny k_philox_words launch: brackets the timed region in rocprofv3 kernel traces."""
    from hyperscalees_t2i_amd import kernels as K
    K.philox_words(0xBEEF, 0, 1, torch.device("cuda", torch.cuda.current_device()))


def load_pmc(name: str = "pmc_lora_gemm.json"):
    f = ROOT / "profiles" / name
    if f.exists():
        try:
            return json.loads(f.read_text())
        except Exception:
            return None
    return None


def load_pmc_traffic():
    return load_pmc("pmc_lora_gemm.json")


def mfma_busy_summary():
    """Counter-measured MFMA-busy fraction of the LoRA GEMM variants (profiles/pmc_lora_gemm_mfma.json, written by
    tools/gemm_mfma_summary.py from a separate rocprofv3 --pmc pass: the profiler cannot run inside this process)."""
    d = load_pmc("pmc_lora_gemm_mfma.json")
    if not d:
        return None
    return {"shape": d.get("shape"), "method": d.get("method"),
            "source": "profiles/pmc_lora_gemm_mfma.json",
            "kernels": {k: {kk: v[kk] for kk in ("mfma_busy_frac", "mfma_busy_frac_at_2.4GHz", "clock_GHz",
                                                 "duration_us_median") if kk in v}
                        for k, v in d.get("kernels", {}).items()},
            "note": "SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE x 128 SIMDs per XCD): the share of SIMD-cycles "
                    "with an MFMA executing at the clock the chip held; _at_2.4GHz prices the same MFMA cycles "
                    "against the peak clock (the vendor 2.5 PF figure's)"}


def seeded_valu_summary():
    """Counter-measured VALU issue of the engine-default seeded ES kernels (profiles/pmc_es_seeded_valu.json, written
    by tools/es_valu_summary.py from tools/pmc_es_valu.sh): the factors are regenerated inside perturb / update
    (Philox4x32-10 + Box-Muller), so these launches are priced against the VALU issue rate beside their HBM bytes."""
    d = load_pmc("pmc_es_seeded_valu.json")
    if not d:
        return None
    return {"method": d.get("method"), "source": "profiles/pmc_es_seeded_valu.json", "groups": d.get("groups"),
            "note": "valu_active = SQ_ACTIVE_INST_VALU x 4 / (GRBM_GUI_ACTIVE / 8 x 1024 SIMDs): the share of SIMD-cycles "
                    "issuing VALU work (quarter-rate 32x32->64 multiplies and transcendentals at their cost); "
                    "valu_issue_2 = SQ_INSTS_VALU x 2 cycles / the same: every op at the full wave64 rate; "
                    "valu_active_at_2.4GHz = the VALU-active SIMD-cycles over duration x 2.4 GHz x 1024 SIMDs (the "
                    "peak clock; the GRBM window of a 15-30 us launch includes dispatch overhead)"}


LINE_MAX_BYTES = 4096   # the driver reads the tail of stdout: the headline line stays small
DEFAULT_AUX = ROOT / "gpurun_out" / "bench_aux.json"


def algo_bytes(shape):
    """bf16 X [M,K] + W [K,N] read once + Y [M,N] written once: the GEMM's algorithmic HBM bytes."""
    try:
        M, K, N = (int(v) for v in str(shape).split("x"))
    except (TypeError, ValueError):
        return None
    return 2.0 * (M * K + K * N + M * N)


def _r(x, nd=4):
    return None if x is None else (round(float(x), nd) if isinstance(x, (int, float)) else x)


def compact_line(full: dict, aux_path: str) -> dict:
    """The one stdout line: headline keys, the roofline kernel's own figures and the CPU baseline's
    value / cores / kind / one-line sample.  Everything else (per-kernel tables, in-product mix,
    achievable peaks, per-variant MFMA-busy) lives in the aux JSON named in `details`."""
    roof = full.get("roofline") or {}
    mb = roof.get("mfma_busy") or {}
    dom = str(roof.get("kernel", "")).split(" ")[0]
    busy = None
    for k, v in (mb.get("kernels") or {}).items():
        if k.replace(" ", "") == dom.replace(" ", ""):
            busy = v.get("mfma_busy_frac")
    mix = roof.get("in_product_mix") or {}
    croof = {"kernel": dom, "bound": roof.get("bound"), "achieved": _r(roof.get("achieved"), 2),
             "peak": roof.get("peak"), "unit": roof.get("unit"), "frac": _r(roof.get("frac")),
             "traffic": _r(roof.get("traffic"), 0), "algorithmic_bytes": _r(roof.get("algorithmic_bytes"), 0),
             "avg_launch_us": _r(roof.get("avg_launch_us"), 2), "launches": roof.get("launches"),
             "flops_per_launch": _r(roof.get("flops_per_launch"), 0), "mfma_busy": _r(busy),
             "in_product_mix_frac": _r(mix.get("frac"))}
    cpu = full.get("cpu_baseline")
    ccpu = None
    if cpu:
        sample = " ".join(str(cpu.get("sample", "")).split())
        ccpu = {"value": _r(cpu.get("value"), 6), "unit": cpu.get("unit"), "cores": cpu.get("cores"),
                "kind": cpu.get("kind"), "sample": sample[:700]}
    keep = ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
            "vs_baseline", "dtype", "data", "config")
    out = {k: full.get(k) for k in keep}
    out["roofline"] = croof
    out["cpu_baseline"] = ccpu
    for k in ("theta_replicas_identical", "theta_final_sha16"):
        if k in full:
            out[k] = full[k]
    out["details"] = aux_path
    return out


def emit(full: dict, gemm: dict, args) -> None:
    """Write the full record to --aux-out (default gpurun_out/bench_aux.json), then print the compact
    headline line LAST on stdout so a tail reader always sees it whole."""
    aux = Path(args.aux_out) if args.aux_out else DEFAULT_AUX
    try:
        aux.parent.mkdir(parents=True, exist_ok=True)
        aux.write_text(json.dumps({"line": full, "gemm": gemm}, indent=1, default=str))
        aux_s = os.path.relpath(aux, ROOT) if aux.is_absolute() else str(aux)
    except OSError as e:
        log(f"aux write failed: {e}")
        aux_s = None
    line = json.dumps(compact_line(full, aux_s), separators=(",", ":"))
    assert len(line.encode()) <= LINE_MAX_BYTES, len(line)
    sys.stderr.flush()
    print(line, flush=True)


def main():
    args = parse()
    rank, world, local = dist_setup(args)
    if rank == 0:
        start_heartbeat()
    device = torch.device(f"cuda:{local}")
    from hyperscalees_t2i_amd.lora import GemmTimer

    backend, engine, noiser, theta, pop = build(args, world, rank, device)
    log(f"rank {rank}: built (pop {pop}, D {noiser.num_params})")
    guidance = backend.cfg.guidance_scale
    S_log = []   # (epoch seed, gathered S [pop, m]) per epoch: the aux record's per-epoch S digests
    for w in range(args.warmup):
        theta, st_w = engine.step(theta, seed=w, guidance_scale=guidance)
        S_log.append((w, st_w.get("_S")))
        torch.cuda.synchronize()
        log(f"rank {rank}: warmup epoch {w} done")
    torch.cuda.synchronize()
    barrier(world)
    torch.cuda.synchronize()
    marker()  # rocprof trace marker: timed region begins (tools/trace_window.py)
    t0 = time.perf_counter()
    for s in range(args.steps):
        theta, stats = engine.step(theta, seed=args.warmup + s, guidance_scale=guidance)
        S_log.append((args.warmup + s, stats.get("_S")))   # host copy the step already made
    torch.cuda.synchronize()
    barrier(world)
    torch.cuda.synchronize()
    elapsed = max_over_ranks(time.perf_counter() - t0, world)
    log(f"rank {rank}: timed {args.steps} epochs in {elapsed:.3f}s")
    marker()  # timed region ends
    # Roofline window: the same epochs again with the LoRA GEMM instrumented (HIP events on its launch
    # stream around each kernel), outside the headline timed region so the instrumentation cannot
    # touch `value`.  Its wall time is reported next to the headline one.
    n_roof = max(1, min(args.steps, 5))
    GemmTimer.reset(True)
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    for s in range(n_roof):
        theta, st_r = engine.step(theta, seed=args.warmup + args.steps + s, guidance_scale=guidance)
        S_log.append((args.warmup + args.steps + s, st_r.get("_S")))
    torch.cuda.synchronize()
    roof_ms_per_step = 1e3 * (time.perf_counter() - t1) / n_roof
    GemmTimer.active = False
    replicas_identical = None
    if world > 1:  # theta' must be bit-identical on every rank (outside the timed region)
        from hyperscalees_t2i_amd.es_step import verify_theta_replicas
        try:
            verify_theta_replicas(theta, engine.dist)
            replicas_identical = True
        except RuntimeError as e:  # reported in the line, not fatal: the throughput was still measured
            log(f"rank {rank}: {e}")
            replicas_identical = False
    gemm = GemmTimer.summary()
    # one extra instrumented epoch for the per-phase breakdown (not part of the timed region)
    from hyperscalees_t2i_amd.kernels import OpTimer
    OpTimer.reset(True)
    theta, st_t = engine.step(theta, seed=10_000, guidance_scale=guidance, timing=True)
    S_log.append((10_000, st_t.get("_S")))
    OpTimer.active = False
    # final theta (after every epoch this run made): equal across ranks and to a single-process run of
    # the same total population (tests/test_gpu_bench_dist.py compares them)
    import hashlib
    theta_sha16 = hashlib.sha256(theta.detach().cpu().numpy().tobytes()).hexdigest()[:16]
    phases = dict(engine.timings)
    S_epochs = [{"seed": sd, "sha16": hashlib.sha256(S.numpy().tobytes()).hexdigest()[:16], "S": S.tolist()}
                for sd, S in S_log if S is not None]
    model_kernels = OpTimer.summary(HBM_PEAK_GBPS)
    from hyperscalees_t2i_amd.measure import aux_kernel_rooflines
    aux = aux_kernel_rooflines(noiser.layout, pop, engine.lo, engine.hi, device, theta=theta)
    # the same kernels at one GPU's share of configs[2] (pop 64 over 8 GPUs: noise and update over
    # all 32 base samples, perturb of this GPU's 8 members) — the sizes the node-level metric runs
    aux64 = None
    if pop != 64 and not args.small and args.workload == "sana":
        aux64 = aux_kernel_rooflines(noiser.layout, 64, 0, args.pop_per_gpu, device, theta=theta)
    # the same ES kernels at one GPU's share of the other node-level configs' theta layouts:
    # configs[3] Z-Image-Turbo (egg rank 4, pop 128 over 8 GPUs: the larger rank-(N*r) update) and
    # configs[4] Infinity-8B (pop 32 over 8 GPUs); the model hosts themselves are out of scope
    aux_cfg = None
    if not args.small and args.workload == "sana":
        from hyperscalees_t2i_amd.kernels import ThetaLayout
        from hyperscalees_t2i_amd.model_shapes import infinity_lora_shapes, zimage_turbo_lora_shapes
        aux_cfg = {
            "configs3_zimage_turbo_r4_pop128": aux_kernel_rooflines(ThetaLayout(zimage_turbo_lora_shapes(), 4), 128, 0,
                                                                    16, device),
            "configs4_infinity_8b_pop32": aux_kernel_rooflines(ThetaLayout(infinity_lora_shapes(), 1), 32, 0, 4,
                                                               device)}

    peaks = None
    if rank == 0 and not args.small:   # achievable peaks on this box next to the vendor ones
        from hyperscalees_t2i_amd.measure import achievable_peaks
        peaks = achievable_peaks(device)
    value = pop * args.steps / elapsed
    variants = {k: v for k, v in gemm.items() if k != "all" and "tflops" in v}
    dom_name = max(variants, key=lambda k: variants[k]["total_ms"]) if variants else "all"
    dom = gemm.get(dom_name, {"launches": 0, "flops": 0.0, "avg_us": float("nan"), "tflops": float("nan")})
    achieved = dom["tflops"]
    # the whole launch mix the epochs run (every LoRA'd linear's GEMM, fused epilogue ops included): what
    # the product path achieves on average, next to the dominant kernel's own rate
    mix = gemm.get("all")
    in_product = None
    if mix:
        in_product = {"tflops": mix["tflops"], "frac": mix["tflops"] / BF16_DENSE_PEAK_TFLOPS,
                      "launches_per_epoch": mix["launches"] / max(n_roof, 1),
                      "gemm_ms_per_epoch": mix["total_ms"] / max(n_roof, 1),
                      "epilogue_bytes_per_epoch": mix["epi_bytes"] / max(n_roof, 1),
                      "variants": {k: {kk: v[kk] for kk in ("launches", "avg_us", "tflops", "epi_bytes", "shape")
                                       if kk in v} for k, v in variants.items()},
                      "note": "GEMM kernels only (projections separate); epi_bytes = the fused op's HBM bytes beyond "
                              "the bf16 y write (fp32 residual stream read + write + shadow for res32 / gated32)"}
    # PMC traffic was collected on the Sana epoch's LoRA-GEMM launch mix (tools/lora_epoch_driver.py):
    # it belongs to that workload's line only
    pmc = load_pmc_traffic() if args.workload == "sana" and not args.small else None
    # the roofline kernel's own launch shape (131072 x 2240 x 2240, r 2; tools/gemm_mfma_driver.py), preferred
    pmc_shape = load_pmc("pmc_lora_gemm_rooflineshape.json") if args.workload == "sana" and not args.small else None
    roofline = {"kernel": f"{dom_name} (population LoRA GEMM + fused LoRA epilogue)", "bound": "mfma",
                "achieved": achieved, "peak": BF16_DENSE_PEAK_TFLOPS, "unit": "TFLOP/s",
                "frac": achieved / BF16_DENSE_PEAK_TFLOPS,
                "traffic": (pmc_shape or pmc or {}).get("hbm_bytes_per_launch"),
                "traffic_measured_on": (("the roofline kernel's launch shape, 131072 x 2240 x 2240 r 2 "
                                         "(tools/gemm_mfma_driver.py; FETCH_SIZE x 2 + WRITE_SIZE per launch); "
                                         "profiles/pmc_lora_gemm_rooflineshape.json") if pmc_shape else
                                        ("one epoch's LoRA-GEMM launch mix x2 (tools/lora_epoch_driver.py: every Sana "
                                         "LoRA'd linear's shape, no epilogue op); profiles/pmc_lora_gemm.json")
                                        if pmc else None),
                "traffic_launch_mix": (pmc or {}).get("hbm_bytes_per_launch"),
                "mfma_busy": mfma_busy_summary() if args.workload == "sana" and not args.small else None,
                "algorithmic_bytes": algo_bytes(dom.get("shape")),
                "launches": dom["launches"], "avg_launch_us": dom["avg_us"],
                "flops_per_launch": dom["flops"] / max(dom["launches"], 1),
                "window": {"epochs": n_roof, "ms_per_step": roof_ms_per_step,
                           "note": "HIP events on the launch stream around each kernel of the product path (fused "
                                   "epilogues kept; each linear's projection and GEMM as their two launches); "
                                   "epochs right after the timed region"},
                "in_product_mix": in_product, "achievable_peaks": peaks,
                "frac_of_achievable": (achieved / max(peaks["bf16_gemm_tflops_hipblaslt"],
                                                      peaks["bf16_gemm_tflops_eggroll"]) if peaks else None)}
    for k, v in gemm.items():  # the projection pre-passes (HBM-bound) join the aux kernel table
        if k.startswith("k_lora_project"):
            key = "lora_project_multi" if k.endswith("multi") else "lora_project"
            aux[key] = {"us": v["avg_us"], "bytes": v["bytes"] / v["launches"], "GBps": v["GBps"],
                        "frac": v["GBps"] / HBM_PEAK_GBPS, "launches": v["launches"]}
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline and args.workload == "sana":
        from oracle import cpu_baseline
        cpu = cpu_baseline.run()
        log(f"cpu baseline: {cpu['value']:.4g} member-evals/s on {cpu['cores']} threads ({cpu.pop('wall_s'):.1f}s)")
    if rank == 0 and args.workload == "zimage":
        c = backend.cfg
        line = {
            "metric": "ES member-evals/sec Z-Image-Turbo 384px egg_rank=4 (BASELINE configs[3], pop 128 over 8 GPUs)",
            "value": value, "unit": "member-evals/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": 1e3 * elapsed / args.steps, "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "dtype": "bf16",
            "data": "synthetic (random-init Z-Image-Turbo 6B / FLUX VAE / CLIP weights, synthetic Qwen3 prompt embeds)",
            "config": {"workload": "tiny-arch smoke (INVALID as metric)" if args.small else "zimage_turbo_384px_es_epoch",
                       "pop_per_gpu": args.pop_per_gpu, "pop_total": pop,
                       "images_per_member": c.prompts_per_gen * c.batches_per_gen, "resolution_px": c.width_px,
                       "steps": c.num_inference_steps, "guidance": c.guidance_scale, "egg_rank": 4, "lora_r": c.lora_r,
                       "lora_alpha": c.lora_alpha, "theta_D": noiser.num_params,
                       "parallelism": f"member-shard x{world} (S all-gather)"},
            "roofline": roofline, "cpu_baseline": None, "phases_ms": phases, "aux_kernels": aux,
            "model_kernels": model_kernels,
        }
    elif rank == 0 and args.workload == "infinity":
        c = backend.cfg
        line = {
            "metric": "ES member-evals/sec Infinity-8B 512px (BASELINE configs[4], pop 32 over 8 GPUs)",
            "value": value, "unit": "member-evals/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": 1e3 * elapsed / args.steps, "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "dtype": "bf16",
            "data": "synthetic (random-init Infinity-8B / BSQ-VAE decoder / CLIP weights, synthetic T5 prompt features)",
            "config": {"workload": "tiny-arch smoke (INVALID as metric)" if args.small else "infinity_8b_512px_es_epoch",
                       "pop_per_gpu": args.pop_per_gpu, "pop_total": pop,
                       "images_per_member": c.prompts_per_gen * c.batches_per_gen, "pn": c.pn,
                       "scales": len(backend.es_model.scale_schedule), "cfg": c.cfg_list, "tau": c.tau_list,
                       "top_k": c.top_k, "top_p": c.top_p, "micro_batch": c.micro_batch, "egg_rank": 1,
                       "lora_r": c.lora_r, "lora_alpha": c.lora_alpha, "lora_targets": c.lora_target_modules,
                       "theta_D": noiser.num_params, "parallelism": f"member-shard x{world} (S all-gather)"},
            "roofline": roofline, "cpu_baseline": None, "phases_ms": phases, "aux_kernels": aux,
            "model_kernels": model_kernels,
        }
    elif rank == 0 and args.workload == "var_d16":
        c = backend.cfg
        line = {
            "metric": "ES member-evals/sec VAR-d16 class-conditional 256px pop=4 (BASELINE configs[0] on the GPU path)",
            "value": value, "unit": "member-evals/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": 1e3 * elapsed / args.steps, "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "dtype": "bf16",
            "data": "synthetic (random-init VAR-d16 / VQVAE ch160 / CLIP weights; no checkpoint offline)",
            "config": {"workload": "tiny-arch smoke (INVALID as metric)" if args.small else "var_d16_256px_es_epoch",
                       "pop_per_gpu": args.pop_per_gpu, "pop_total": pop,
                       "images_per_member": c.classes_per_gen * c.batches_per_gen, "classes_per_gen": c.classes_per_gen,
                       "batches_per_gen": c.batches_per_gen, "cfg": c.guidance_scale, "top_k": c.top_k, "top_p": c.top_p,
                       "egg_rank": 1, "lora_r": c.lora_r, "lora_alpha": c.lora_alpha, "theta_D": noiser.num_params,
                       "parallelism": f"member-shard x{world} (S all-gather)"},
            "roofline": roofline, "cpu_baseline": None, "phases_ms": phases, "aux_kernels": aux,
            "model_kernels": model_kernels,
        }
    elif rank == 0:
        line = {
            "metric": METRIC, "value": value, "unit": "member-evals/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": 1e3 * elapsed / args.steps, "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "bf16",
            "data": "synthetic (random-init Sana-Sprint-1.6B/DC-AE/CLIP-H/CLIP-B weights, synthetic prompt embeds)",
            "config": {"workload": ("tiny-arch smoke (INVALID as metric)" if args.small else
                                    "sana_sprint_1.6b_onestep_1024px_es_epoch"),
                       "pop_per_gpu": args.pop_per_gpu, "pop_total": pop, "images_per_member": 16,
                       "prompts_per_gen": 4, "batches_per_gen": 4, "resolution_px": 32 * args.latent,
                       "egg_rank": 1, "lora_r": 2, "lora_alpha": 8, "theta_D": noiser.num_params,
                       "antithetic": True, "promptnorm": True, "reward": "PickScore(CLIP-H/14)+CLIP-B/32",
                       "parallelism": f"member-shard x{world} (S all-gather)"},
            "roofline": roofline,
            "cpu_baseline": cpu,
            "theta_replicas_identical": replicas_identical,
            "theta_final_sha16": theta_sha16,
            "S_epochs": S_epochs,
            "phases_ms": phases,
            "aux_kernels": aux,
            "aux_kernels_pop64_per_gpu": aux64,
            "aux_kernels_other_configs_per_gpu": aux_cfg,
            "aux_kernels_seeded_valu": seeded_valu_summary() if not args.small else None,
            "model_kernels": model_kernels,
        }
    if rank == 0:
        emit(line, gemm, args)
    if world > 1:
        import torch.distributed as dist
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
