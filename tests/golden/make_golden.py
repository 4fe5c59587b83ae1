"""Generate golden vectors from the REFERENCE implementation (run in the build container only).

    python tests/golden/make_golden.py          # needs /root/reference (read-only mount)

Imports the reference's own `utills.py` (amit154154/HyperscaleES_T2I) and records, for small
seeded inputs, the outputs of the functions on the ES hot path.  The random factors that
`EggRollNoiser._sample_low_rank_block` draws with `torch.randn` (utills.py:59-65) are captured
by wrapping torch.randn, so the fixtures double as NOISE-INJECTION vectors: feeding the
captured factors to our kernels must reproduce the reference eps exactly.
Fixtures are data only (inputs + expected outputs), written to tests/golden/*.npz.
The GPU box never runs this script and never reads /root/reference.
"""
from __future__ import annotations

import math
import sys
from pathlib import Path

import numpy as np
import torch

REF = Path("/root/reference")
OUT = Path(__file__).resolve().parent


def load_reference():
    if not (REF / "utills.py").exists():
        raise SystemExit("reference not mounted at /root/reference")
    sys.path.insert(0, str(REF))
    import utills  # noqa: E402  (reference module)
    return utills


class RandnRecorder:
    """Wraps torch.randn; records every tensor drawn (in call order)."""

    def __init__(self):
        self.calls = []
        self._orig = torch.randn

    def __enter__(self):
        orig = self._orig

        def rec(*a, **k):
            t = orig(*a, **k)
            self.calls.append(t.detach().clone())
            return t

        torch.randn = rec
        return self

    def __exit__(self, *exc):
        torch.randn = self._orig


SHAPE_SETS = {
    # LoRA-like: lora_A [r_l, in], lora_B [out, r_l] pairs + a 1-D param (dense fallback)
    "lora_small": [(2, 12), (10, 2), (2, 7), (5, 2)],
    "mixed": [(3, 4), (6,), (2, 9), (9, 2), (1, 1)],
}


def gen_eps(u):
    recs = {}
    idx = 0
    for sname, shapes in SHAPE_SETS.items():
        for pop in (1, 2, 3, 4, 5, 8):
            for rank in (1, 2, 4):
                for anti in (False, True):
                    for seed in (0, 3):
                        torch.manual_seed(seed)
                        noiser = u.EggRollNoiser([torch.Size(s) for s in shapes], sigma=0.01, lr_scale=0.1,
                                                 rank=rank, use_antithetic=anti)
                        with RandnRecorder() as rr:
                            eps = noiser.sample_eps(pop, "cpu")
                        base_pop = (pop // 2 + pop % 2) if anti else pop
                        # flatten captured factors into our per-base-sample layout
                        parts = []
                        ci = 0
                        for s in shapes:
                            if len(s) == 2:
                                a, b = rr.calls[ci], rr.calls[ci + 1]
                                ci += 2
                                parts.append(a.reshape(base_pop, -1))
                                parts.append(b.reshape(base_pop, -1))
                            else:
                                parts.append(rr.calls[ci].reshape(base_pop, -1))
                                ci += 1
                        assert ci == len(rr.calls)
                        factors = torch.cat(parts, dim=1)
                        theta = torch.randn(noiser.num_params, generator=torch.Generator().manual_seed(100 + idx))
                        k = pop - 1
                        theta_k = theta + noiser.sigma * eps[k]
                        key = f"{sname}_p{pop}_r{rank}_a{int(anti)}_s{seed}"
                        recs[key + "/factors"] = factors.numpy()
                        recs[key + "/eps"] = eps.numpy()
                        recs[key + "/theta"] = theta.numpy()
                        recs[key + "/theta_last"] = theta_k.numpy()
                        idx += 1
    recs["meta/shape_sets"] = np.array(repr(SHAPE_SETS))
    np.savez_compressed(OUT / "g1_eps.npz", **recs)
    return len(recs)


def gen_fitness(u):
    recs = {}
    g = torch.Generator().manual_seed(7)
    cases = {}
    for n in (1, 2, 3, 4, 8, 64, 128):
        for m in (1, 4):
            cases[f"rand_n{n}_m{m}"] = torch.randn(n, m, generator=g) * 3 + 20
    cases["tied_rows"] = torch.tensor([[1.0, 2.0], [1.0, 2.0], [0.5, 3.0], [1.0, 2.0]])
    cases["const"] = torch.full((6, 4), 21.5)
    t = torch.randn(8, 4, generator=g)
    t[3, 1] = float("nan")
    cases["nan_one"] = t
    t = torch.randn(8, 4, generator=g)
    t[:, 0] = float("inf")
    cases["inf_col"] = t
    t = torch.randn(5, 3, generator=g)
    cases["ints"] = torch.round(t * 4)
    for name, S in cases.items():
        scores, mu, sb = u.paper_prompt_normalized_scores(S)
        recs[f"{name}/S"] = S.numpy()
        recs[f"{name}/pn_scores"] = scores.numpy()
        recs[f"{name}/pn_mu"] = mu.numpy()
        recs[f"{name}/pn_sigma_bar"] = np.array(sb.item(), np.float32)
        recs[f"{name}/mean_scores"] = S.mean(dim=1).numpy()
        for tag, sc in (("pn", scores), ("mean", S.mean(dim=1))):
            fin = torch.isfinite(sc)
            recs[f"{name}/{tag}_finite"] = fin.numpy()
            if fin.any():
                recs[f"{name}/{tag}_fitness"] = u.standardize_fitness(sc[fin]).numpy()
            if fin.all():
                recs[f"{name}/{tag}_order"] = torch.sort(sc, stable=True)[1].numpy()
    # z-score edge cases (utills.py:168-178)
    for name, r in {"z_one": torch.tensor([3.0]), "z_two": torch.tensor([1.0, 2.0]),
                    "z_const": torch.full((5,), 2.0), "z_rand": torch.randn(33, generator=g)}.items():
        import warnings
        with warnings.catch_warnings():
            warnings.simplefilter("ignore")
            recs[f"{name}/r"] = r.numpy()
            recs[f"{name}/f"] = u.standardize_fitness(r).numpy()
    np.savez_compressed(OUT / "g2_fitness.npz", **recs)
    return len(recs)


def gen_update(u):
    recs = {}
    g = torch.Generator().manual_seed(11)
    shapes = SHAPE_SETS["lora_small"]
    D = sum(int(np.prod(s)) for s in shapes)
    for pop in (2, 5, 8):
        for caps in ((0.0, 0.0), (0.0, 40.0), (1e-3, 40.0), (0.0, 1.0), (5e-4, 1.0)):
            torch.manual_seed(pop)
            noiser = u.EggRollNoiser([torch.Size(s) for s in shapes], sigma=0.01, lr_scale=0.1, rank=1,
                                     use_antithetic=True)
            eps = noiser.sample_eps(pop, "cpu")
            theta = torch.randn(D, generator=g) * 0.3
            raw = torch.randn(pop, generator=g)
            f = noiser.convert_fitnesses(raw)
            after = noiser.do_update(theta, eps, f)
            after_s = u.cap_step_norm(theta, after, caps[0])
            after_t = u.cap_theta_norm(after_s, caps[1])
            key = f"p{pop}_ms{caps[0]}_mt{caps[1]}"
            recs[key + "/theta"] = theta.numpy()
            recs[key + "/eps"] = eps.numpy()
            recs[key + "/raw"] = raw.numpy()
            recs[key + "/f"] = f.numpy()
            recs[key + "/after_update"] = after.numpy()
            recs[key + "/after_caps"] = after_t.numpy()
    np.savez_compressed(OUT / "g4_update.npz", **recs)
    return len(recs)


def gen_indices(u):
    recs = {}
    for P in (4, 8, 1631):
        for k in (1, 2, 4, 7):
            rows = []
            for seed in range(100):
                rows.append(u.sample_indices_unique(seed, P, k))
            recs[f"P{P}_k{k}"] = np.array(rows, np.int64)
    recs["repeat_4x3"] = np.array(u.repeat_batches([3, 1, 2, 0], 3), np.int64)
    np.savez_compressed(OUT / "g5_indices.npz", **recs)
    return len(recs)


def ref_step_sampling_info(u, seed, P, prompts_per_gen, batches_per_gen, max_log_batches, prompts_list=None):
    """SanaBackend.step_sampling_info (es_backend.py:234-263) composed from the reference's own
    utills functions exactly as that method does (es_backend.py itself needs diffusers/peft)."""
    unique_ids = u.sample_indices_unique(seed=seed, total=P, k=prompts_per_gen)
    flat_ids = u.repeat_batches(unique_ids, repeats=batches_per_gen)
    pid_to_j = {pid: j for j, pid in enumerate(unique_ids)}
    m = len(unique_ids)
    unique_texts = [prompts_list[pid] if prompts_list is not None else f"prompt_{pid}" for pid in unique_ids]
    flat_texts = [(prompts_list[pid] if prompts_list is not None else f"prompt_{pid}") for pid in flat_ids]
    log_batches = int(max(0, min(max_log_batches, batches_per_gen)))
    return dict(unique_ids=unique_ids, flat_ids=flat_ids, unique_texts=unique_texts, flat_texts=flat_texts,
                pid_to_j=pid_to_j, m=m, total_imgs_per_indiv=len(flat_ids),
                total_imgs_for_logging=log_batches * m, log_batches=log_batches)


def ref_var_classes(seed, allowed, classes_per_gen, num_classes_total=1000):
    """VarBackend._sample_classes_unique (es_backend.py:377-396), restated line by line (the method
    lives on a class whose module needs peft; the arithmetic is numpy only)."""
    rng = np.random.RandomState(int(seed))
    if allowed is None or allowed == "all":
        pool = np.arange(num_classes_total, dtype=np.int64)
    else:
        pool = np.array(list(allowed), dtype=np.int64)
        pool = np.unique(pool)
        pool = pool[(pool >= 0) & (pool < num_classes_total)]
        if pool.size == 0:
            pool = np.arange(num_classes_total, dtype=np.int64)
    m = int(classes_per_gen)
    return rng.choice(pool, size=m, replace=False).tolist()


def gen_sampling_info(u):
    """g5b: the reference step_sampling_info dict for seeds 0-99 (P in {4, 1631}) and the VAR class
    sampler; integer fields as arrays, pid_to_j as (pid, j) pairs, texts joined with '\x1f'."""
    recs = {}
    for P in (4, 1631):
        for k in (1, 2, 4):
            for R in (1, 4):
                for mlb in (0, 1, 2, 5):
                    prompts = [f"prompt text {i}" for i in range(P)] if (P == 4 and mlb == 1) else None
                    rows = {f: [] for f in ("unique_ids", "flat_ids", "pid_to_j", "scalars", "texts")}
                    for seed in range(100):
                        d = ref_step_sampling_info(u, seed, P, k, R, mlb, prompts)
                        rows["unique_ids"].append(d["unique_ids"])
                        rows["flat_ids"].append(d["flat_ids"])
                        rows["pid_to_j"].append(sorted(d["pid_to_j"].items()))
                        rows["scalars"].append([d["m"], d["total_imgs_per_indiv"], d["total_imgs_for_logging"],
                                                d["log_batches"]])
                        rows["texts"].append("\x1f".join(d["unique_texts"] + d["flat_texts"]))
                    key = f"P{P}_k{k}_R{R}_L{mlb}" + ("_named" if prompts else "")
                    for f in ("unique_ids", "flat_ids", "pid_to_j", "scalars"):
                        recs[f"{key}/{f}"] = np.array(rows[f], np.int64)
                    recs[f"{key}/texts"] = np.array(rows["texts"])
    for allowed, tag in ((None, "all"), ([3, 3, 17, 999, 1000, -1, 42, 7, 17, 500], "list")):
        for mcls in (1, 4):
            recs[f"var_{tag}_m{mcls}"] = np.array([ref_var_classes(s, allowed, mcls) for s in range(100)], np.int64)
    np.savez_compressed(OUT / "g5b_sampling_info.npz", **recs)
    return len(recs)


def gen_s_aggregation():
    """g9: unifed_es.py:165-215 restated literally (per-image loop, per_prompt_comb lists,
    torch.stack(...).mean()) on seeded per-image rewards, for repeat orders the reference produces and
    for a shuffled flat order (pid_to_j does the grouping, not the position)."""
    recs = {}
    g = torch.Generator().manual_seed(31)
    cases = {"m4_R4": ([5, 2, 9, 0] * 4), "m2_R3": ([1, 0] * 3), "m3_R1": [2, 0, 1],
             "shuffled": [3, 1, 3, 2, 1, 2, 3, 1, 2], "ragged": [4, 4, 4, 8, 8]}
    for name, flat_ids in cases.items():
        unique = list(dict.fromkeys(flat_ids))
        pid_to_j = {pid: j for j, pid in enumerate(unique)}
        m, pop, B = len(unique), 3, len(flat_ids)
        rew = {k: torch.randn(pop, B, generator=g) * 2 + 20 for k in
               ("combined", "clip_aesthetic", "clip_text", "no_artifacts", "pickscore")}
        S = torch.empty((pop, m))
        raw = torch.empty((pop, 5))
        for k in range(pop):
            per_prompt = [[] for _ in range(m)]
            alls = {key: [] for key in rew}
            for idx in range(B):
                j = pid_to_j[int(flat_ids[idx])]
                per_prompt[j].append(rew["combined"][k, idx].float())
                for key in rew:
                    alls[key].append(rew[key][k, idx].float())
            for j in range(m):
                S[k, j] = torch.stack(per_prompt[j]).mean()
            for c, key in enumerate(("combined", "clip_aesthetic", "clip_text", "no_artifacts", "pickscore")):
                raw[k, c] = torch.stack(alls[key]).mean()
        recs[f"{name}/flat_ids"] = np.array(flat_ids, np.int64)
        recs[f"{name}/unique_ids"] = np.array(unique, np.int64)
        for key, v in rew.items():
            recs[f"{name}/rew_{key}"] = v.numpy()
        recs[f"{name}/S"] = S.numpy()
        recs[f"{name}/raw"] = raw.numpy()
    np.savez_compressed(OUT / "g9_s_aggregation.npz", **recs)
    return len(recs)


TINY_ARCH = dict(num_attention_heads=4, attention_head_dim=32, num_layers=2, num_cross_attention_heads=2,
                 cross_attention_head_dim=64, caption_channels=2304)


def gen_member_eval_injection(u):
    """g10: reference EggRollNoiser factors captured on the LoRA theta layout of the tiny Sana
    architecture the GPU parity tests build (tests/test_gpu_parity_fp32.py), pop 8, egg rank 1,
    antithetic, for sigma 1e-2 and 0.5: the injected noise of the bf16-vs-fp32 member-eval test."""
    sys.path.insert(0, str(OUT.parent.parent))
    from hyperscalees_t2i_amd.sana import SanaArch, sana_lora_shapes
    shapes = sana_lora_shapes(SanaArch(**TINY_ARCH))
    recs = {"shapes": np.array(shapes, np.int64)}
    for seed, sigma in ((0, 1e-2), (1, 0.5)):
        torch.manual_seed(seed)
        noiser = u.EggRollNoiser([torch.Size(s) for s in shapes], sigma=sigma, lr_scale=0.1, rank=1,
                                 use_antithetic=True)
        with RandnRecorder() as rr:
            eps = noiser.sample_eps(8, "cpu")
        parts = [t.reshape(4, -1) for t in rr.calls]
        key = f"s{seed}"
        recs[key + "/factors"] = torch.cat(parts, dim=1).numpy()
        recs[key + "/eps"] = eps.numpy()
        recs[key + "/sigma"] = np.array(sigma, np.float32)
    np.savez_compressed(OUT / "g10_member_eval_injection.npz", **recs)
    return len(recs)


def gen_member_eval_fullsize(u):
    """g12: reference EggRollNoiser factors captured on the FULL Sana-Sprint 1.6B LoRA theta layout
    (SanaArch() defaults: 168 targets, 336 matrices, D = 1,515,456; LoRA r 2), pop 2 (one antithetic
    pair = one base sample), egg rank 1, sigma 1e-2 — the injected noise of the full-size bf16-vs-fp32
    member-eval test (tests/test_gpu_parity_fullsize.py).  eps itself (2 x D fp32) is not stored: the
    test checks its reproduction through a sha256 of member 0's eps bytes plus 4096 sampled values."""
    sys.path.insert(0, str(OUT.parent.parent))
    import hashlib
    from hyperscalees_t2i_amd.sana import SanaArch, sana_lora_shapes
    shapes = sana_lora_shapes(SanaArch())
    torch.manual_seed(12)
    noiser = u.EggRollNoiser([torch.Size(s) for s in shapes], sigma=1e-2, lr_scale=0.1, rank=1,
                             use_antithetic=True)
    with RandnRecorder() as rr:
        eps = noiser.sample_eps(2, "cpu")
    assert torch.equal(eps[1], -eps[0])
    parts = [t.reshape(1, -1) for t in rr.calls]
    idx = torch.randperm(eps.shape[1], generator=torch.Generator().manual_seed(3))[:4096].sort()[0]
    recs = {"shapes": np.array(shapes, np.int64), "factors": torch.cat(parts, dim=1).numpy(),
            "sigma": np.array(1e-2, np.float32), "eps0_idx": idx.numpy(), "eps0_at_idx": eps[0, idx].numpy(),
            "eps0_sha256": np.array(hashlib.sha256(eps[0].contiguous().numpy().tobytes()).hexdigest())}
    np.savez_compressed(OUT / "g12_member_eval_fullsize.npz", **recs)
    return len(recs)


VAR_TARGETS = ["mat_qkv", "proj", "fc1", "fc2", "ada_lin.1", "head_nm.ada_lin.1", "head"]  # unifed_es.py:406


def gen_var():
    """g8: BASELINE configs[0] (VAR-d16, LoRA r 4 / alpha 16, unifed_es.py:403-406) from the reference's
    own VAR_models (importable here): the theta layout (PEFT suffix matching of the targets over
    var.named_modules(), lora_A [r, in] then lora_B [out, r] per target) and LoRA'd-linear
    activations of one class-conditional generation at seeded init.  build_vae_var leaves the VQVAE
    weights uninitialised (NaN images), so they are initialised explicitly (seeded
    N(0, 1/fan_in)).  Per distinct linear shape: 64 input rows of the largest call (the last scale,
    CFG-doubled), the first 64 output features of W / bias, the module's own fp32 output on those
    rows, seeded LoRA factors and the PEFT-formula output in fp64 on the bf16-rounded operands."""
    sys.path.insert(0, str(REF))
    import torch.nn as nn
    from VAR_models import build_vae_var
    torch.manual_seed(0)
    vae, var = build_vae_var(device="cpu", depth=16, flash_if_available=False, fused_if_available=False)
    g = torch.Generator().manual_seed(1)
    with torch.no_grad():
        for name, p in vae.named_parameters():
            if p.dim() > 1:
                p.copy_(torch.randn(p.shape, generator=g) / math.sqrt(p[0].numel()))
            elif name.endswith("weight"):
                p.fill_(1.0)
            else:
                p.zero_()
    var.eval()
    targets = [(n, m) for n, m in var.named_modules()
               if isinstance(m, nn.Linear) and any(n == t or n.endswith("." + t) for t in VAR_TARGETS)]
    r = 4
    shapes = []
    for n, m in targets:
        shapes += [(r, m.in_features), (m.out_features, r)]
    recs = {"shapes": np.array(shapes, np.int64), "names": np.array("\x1f".join(n for n, _ in targets))}
    captured = {}

    def hook(name):
        def f(mod, inp, out):
            x = inp[0].detach().reshape(-1, inp[0].shape[-1])
            if name not in captured or x.shape[0] > captured[name][0].shape[0]:
                captured[name] = (x.clone(), out.detach().reshape(-1, out.shape[-1]).clone())
        return f

    hs = [m.register_forward_hook(hook(n)) for n, m in targets]
    with torch.no_grad():
        var.autoregressive_infer_cfg(B=2, label_B=torch.tensor([207, 980]), cfg=1.5, top_k=900, top_p=0.96,
                                     g_seed=0, more_smooth=False)
    for h in hs:
        h.remove()
    seen = set()
    gl = torch.Generator().manual_seed(2)
    for n, m in targets:
        key = (m.in_features, m.out_features)
        if key in seen or n not in captured:
            continue
        seen.add(key)
        x, y = captured[n]
        assert torch.isfinite(x).all() and torch.isfinite(y).all(), n
        rows = torch.linspace(0, x.shape[0] - 1, 64).round().long()
        xs = x[rows].to(torch.bfloat16).float()
        W = m.weight.detach()[:64].to(torch.bfloat16).float()
        b = None if m.bias is None else m.bias.detach()[:64].to(torch.bfloat16).float()
        A = (torch.rand(r, m.in_features, generator=gl) * 2 - 1) / math.sqrt(m.in_features)
        B = torch.randn(64, r, generator=gl) * 0.02
        s = 16.0 / r
        y64 = xs.double() @ W.double().T + (0 if b is None else b.double()) + s * ((xs.double() @ A.double().T) @ B.double().T)
        tag = f"lin_{m.in_features}x{m.out_features}"
        recs[tag + "/x"] = xs.numpy()
        recs[tag + "/W"] = W.numpy()
        if b is not None:
            recs[tag + "/b"] = b.numpy()
        recs[tag + "/A"] = A.numpy()
        recs[tag + "/B"] = B.numpy()
        recs[tag + "/y"] = y64.numpy()
        recs[tag + "/y_module"] = y[rows][:, :64].numpy()      # the VAR module's own fp32 output
        recs[tag + "/meta"] = np.array([x.shape[0], s], np.float64)
    np.savez_compressed(OUT / "g8_var.npz", **recs)
    return len(recs)


def gen_var_model():
    """g11: VAR model-level parity (BASELINE configs[0] path at a tiny size): the reference's own
    VAR_models (depth 2 -> width 128, 2 heads; VQVAE ch 32; V 4096, Cvae 32, the 10 default scales)
    with deterministic synthetic weights (tests/var_weights.py, applied by parameter name) and the
    PEFT LoRA formula y += (alpha/r) (x A^T) B^T hooked onto every target linear (r 4, alpha 16,
    es_backend.py:334-341) from a seeded theta (the mat_qkv hook never fires: basic_var.py:93 calls
    F.linear on mat_qkv.weight, which under PEFT is the base weight — the reference's own semantics).  One autoregressive_infer_cfg(B=2, cfg 4, top_k 900,
    top_p 0.95, g_seed 5) on CPU fp32 records: the sampled token maps of every scale, the CFG logits
    fed to the sampler (exact fp32 for scales 0-3 -> sampler replay; fp16 at <= 8 token positions per
    scale for all scales -> teacher-forced logits check), f_hat and the [0, 1] image."""
    sys.path.insert(0, str(REF))
    sys.path.insert(0, str(OUT.parent))
    import torch.nn as nn
    import torch.nn.functional as F
    import VAR_models.var as var_mod
    from VAR_models import build_vae_var
    from var_weights import TARGETS, TINY, synth_state, synth_theta
    torch.manual_seed(0)
    vae, var = build_vae_var(device="cpu", V=4096, Cvae=32, ch=TINY["vae_ch"], share_quant_resi=4,
                             depth=TINY["depth"], shared_aln=False, attn_l2_norm=True,
                             flash_if_available=False, fused_if_available=False)
    var.eval(), vae.eval()
    dec_keys = [(n, tuple(p.shape)) for n, p in vae.named_parameters()
                if not n.startswith(("encoder.", "quant_conv."))]
    var_keys = [(n, tuple(p.shape)) for n, p in var.named_parameters()]
    with torch.no_grad():
        for mod, keys in ((var, var_keys), (vae, dec_keys)):
            st = synth_state(keys)
            own = dict(mod.named_parameters())
            for n, t in st.items():
                own[n].copy_(t)
    targets = [(n, m) for n, m in var.named_modules()
               if isinstance(m, nn.Linear) and any(n == t or n.endswith("." + t) for t in TARGETS)]
    r, s = TINY["lora_r"], TINY["lora_alpha"] / TINY["lora_r"]
    shapes = []
    for n, m in targets:
        shapes += [(r, m.in_features), (m.out_features, r)]
    theta = synth_theta(shapes)
    off, hooks = 0, []
    for n, m in targets:
        A = theta[off:off + r * m.in_features].view(r, m.in_features)
        off += r * m.in_features
        Bm = theta[off:off + m.out_features * r].view(m.out_features, r)
        off += m.out_features * r
        hooks.append(m.register_forward_hook(
            lambda mod, inp, out, A=A, Bm=Bm: out + s * F.linear(F.linear(inp[0], A), Bm)))
    assert off == theta.numel()
    rec = {"idx": [], "logits": []}
    orig = var_mod.sample_with_top_k_top_p_

    def spy(logits_BlV, **kw):
        rec["logits"].append(logits_BlV.detach().clone())
        idx = orig(logits_BlV, **kw)
        rec["idx"].append(idx[:, :, 0].clone())
        return idx

    cap = {}
    orig_f2i = vae.fhat_to_img

    def f2i(f_hat):
        cap["f_hat"] = f_hat.detach().clone()
        return orig_f2i(f_hat)

    var_mod.sample_with_top_k_top_p_ = spy
    vae.fhat_to_img = f2i
    labels = torch.tensor([3, 980])
    try:
        with torch.no_grad():
            img = var.autoregressive_infer_cfg(B=2, label_B=labels, cfg=4.0, top_k=900, top_p=0.95, g_seed=5,
                                               more_smooth=False)
    finally:
        var_mod.sample_with_top_k_top_p_ = orig
        for h in hooks:
            h.remove()
    out = {"labels": labels.numpy(), "theta": theta.numpy(), "lora_shapes": np.array(shapes, np.int64),
           "var_keys": np.array("\x1f".join(f"{n}:{'x'.join(map(str, sh))}" for n, sh in var_keys)),
           "dec_keys": np.array("\x1f".join(f"{n}:{'x'.join(map(str, sh))}" for n, sh in dec_keys)),
           "meta": np.array([4.0, 900, 0.95, 5], np.float64), "f_hat": cap["f_hat"].numpy(),
           "image": img.to(torch.float16).numpy()}
    for si, (lg, idx) in enumerate(zip(rec["logits"], rec["idx"])):
        out[f"idx{si}"] = idx.numpy().astype(np.int16)
        l = lg.shape[1]
        pos = torch.linspace(0, l - 1, min(8, l)).round().long()
        out[f"pos{si}"] = pos.numpy()
        out[f"logit_sub{si}"] = lg[:, pos].to(torch.float16).numpy()
        if si <= 3:
            out[f"logit_full{si}"] = lg.numpy()
    np.savez_compressed(OUT / "g11_var_model.npz", **out)
    return len(out)


def gen_es_tail(u):
    """unifed_es.py:227-281 composed from the reference's own functions (unifed_es.py itself does
    not import here: wandb / lovely_tensors / peft are absent)."""
    recs = {}
    g = torch.Generator().manual_seed(23)
    shapes = SHAPE_SETS["lora_small"]
    for case, (pop, m, pn, nan_row) in enumerate([(8, 4, True, None), (8, 4, False, None), (7, 2, True, None),
                                                  (8, 4, True, 3), (8, 4, False, 5), (64, 4, True, None)]):
        torch.manual_seed(case)
        noiser = u.EggRollNoiser([torch.Size(s) for s in shapes], sigma=0.01, lr_scale=0.1, rank=1,
                                 use_antithetic=True)
        eps = noiser.sample_eps(pop, "cpu")
        theta = torch.randn(noiser.num_params, generator=g)
        S = torch.randn(pop, m, generator=g) + 21
        if nan_row is not None:
            S[nan_row, 0] = float("nan")
        if pn:
            scores, mu, sb = u.paper_prompt_normalized_scores(S)
        else:
            scores = S.mean(dim=1)
        fin = torch.isfinite(scores)
        key = f"case{case}"
        recs[key + "/S"] = S.numpy()
        recs[key + "/eps"] = eps.numpy()
        recs[key + "/theta"] = theta.numpy()
        recs[key + "/cfg"] = np.array([pop, m, int(pn)], np.int64)
        if not fin.any():  # unifed_es.py:237-240 early return: theta unchanged
            after = theta.clone()
        else:
            if fin.all():
                recs[key + "/order"] = torch.sort(scores)[1].numpy()
            f = noiser.convert_fitnesses(scores[fin])
            after = noiser.do_update(theta, eps[fin], f)
            after = u.cap_step_norm(theta, after, 0.0)
            after = u.cap_theta_norm(after, 40.0)
        recs[key + "/after"] = after.numpy()
        recs[key + "/scores"] = scores.numpy()
    np.savez_compressed(OUT / "g6_es_tail.npz", **recs)
    return len(recs)


def gen_lora(u):
    """PEFT LoRA-linear formula (peft not importable here -> formula-level fixture only)."""
    recs = {}
    g = torch.Generator().manual_seed(5)
    for name, (M, K, N, r) in {"small": (24, 64, 40, 2), "r4": (16, 128, 72, 4)}.items():
        x = torch.randn(M, K, generator=g, dtype=torch.float64)
        W = torch.randn(N, K, generator=g, dtype=torch.float64) * 0.05
        b = torch.randn(N, generator=g, dtype=torch.float64)
        A = torch.randn(r, K, generator=g, dtype=torch.float64) * 0.1
        B = torch.randn(N, r, generator=g, dtype=torch.float64) * 0.1
        s = 8.0 / r
        y = torch.nn.functional.linear(x, W, b) + torch.nn.functional.linear(torch.nn.functional.linear(x, A), B) * s
        for k, v in dict(x=x, W=W, b=b, A=A, B=B, y=y).items():
            recs[f"{name}/{k}"] = v.numpy()
        recs[f"{name}/scale"] = np.array(s)
    np.savez_compressed(OUT / "g7_lora.npz", **recs)
    return len(recs)


if __name__ == "__main__":
    if sys.argv[1:] == ["var_model"]:          # regenerate g11 only
        print("gen_var_model", gen_var_model())
        raise SystemExit(0)
    if sys.argv[1:] == ["fullsize"]:           # regenerate g12 only
        torch.set_num_threads(1)
        print("gen_member_eval_fullsize", gen_member_eval_fullsize(load_reference()))
        raise SystemExit(0)
    u = load_reference()
    torch.set_num_threads(1)
    for fn in (gen_eps, gen_fitness, gen_update, gen_indices, gen_sampling_info, gen_es_tail, gen_lora,
               gen_member_eval_injection, gen_member_eval_fullsize):
        print(fn.__name__, fn(u))
    print("gen_s_aggregation", gen_s_aggregation())
    print("gen_var", gen_var())
    print("gen_var_model", gen_var_model())
