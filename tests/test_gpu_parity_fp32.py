"""bf16 member-eval (the build) vs an fp32 restatement of the reference's per-member path, with
REFERENCE-GENERATED noise injected (north_star: "perturbed activations, rewards and LoRA updates
within a stated bf16/fp32 tolerance, verified by injecting reference-generated noise").

Setup: the tiny Sana / DC-AE / CLIP stack of tests/test_gpu_engine.py (same architecture as the
1.6B model, seeded synthetic weights), pop 8, egg rank 1, antithetic; factors captured from the
reference's own EggRollNoiser (tests/golden/g10, made by make_golden.py from utills.py).
  build:  perturb kernel -> one population-batched bf16 forward on the HIP kernels -> batched
          bf16 rewards -> S (es_step.aggregate_member_rewards) -> fitness kernel -> ranks
  fp32:   theta_k = theta + sigma * eps_k (reference eps) -> oracle/member_eval_fp32.py per member
          (PEFT LoRA formula, same weights upcast, fp16 SCM casts of models/SanaSprint.py) -> S
Measured drift per tensor is asserted against the bounds below; ranks are
compared as the exact order and as Kendall's tau.  Two noise scales: sigma = 1e-2 (the BASELINE
configs) and 0.5 (member differences well above the bf16 noise floor).
"""
import json
import os

import numpy as np
import pytest
import torch

from hyperscalees_t2i_amd import kernels as K
from hyperscalees_t2i_amd.backend import SanaBackend, SanaConfig
from hyperscalees_t2i_amd.es import EggRollNoiser, flatten_params
from hyperscalees_t2i_amd.es_step import aggregate_member_rewards
from hyperscalees_t2i_amd.lora import LoRALinear
from hyperscalees_t2i_amd.rewards import RewardModels
from hyperscalees_t2i_amd.sana import SanaArch
from oracle import eggroll_oracle as O
from oracle import member_eval_fp32 as R

pytestmark = pytest.mark.gpu

TINY = SanaArch(num_attention_heads=4, attention_head_dim=32, num_layers=2, num_cross_attention_heads=2,
                cross_attention_head_dim=64, caption_channels=2304)

# Stated tolerances (bf16 storage / MFMA inputs vs fp32; measured values in DESIGN.md §3).
# s0 = the BASELINE noise scale sigma = 1e-2; s1 = sigma 0.5, where the perturbed network amplifies
# the bf16 rounding with depth (measured round 4: 0.3 % at the first linears -> 8.6 % at block 1's attn1 out)
# while the member spread of S (1.5) still dwarfs |dS| — so ranks must agree there up to near-ties:
# a pair may only swap if its fp32 scores are closer than twice the largest score error (S1_SCORE_ERR
# bounds that error; measured round 4: 0.0036, one pair 0.0024 apart swapped).
BOUNDS = {   # ~1.5x the round-4 measurement (fp32 residual streams in the Sana blocks and DC-AE stages 0-3)
    "s0": {"lora_rel": 6.5e-3,   # every LoRA'd / frozen linear output, ||y - y32|| / ||y32|| (measured 0.43 %)
           "eps_rel": 3e-3,      # transformer output (0.19 %; round 3: 0.56 %)
           "image_rel": 1.25e-2, # decoded image (0.83 %)
           "reward_abs": 0.02,   # per-image combined reward, PickScore scale exp(logit_scale) = 14.3 (0.013)
           "S_abs": 0.0125},     # S[k, j] (0.0081; member spread of S 0.051)
    "s1": {"lora_rel": 0.13, "eps_rel": 0.029, "image_rel": 0.03, "reward_abs": 0.04, "S_abs": 0.022},
}
S1_SCORE_ERR = 0.006
KEYS = ("lora_rel", "eps_rel", "image_rel", "reward_abs", "S_abs")
# test_rank_fidelity_over_seeds (sigma 1e-2, 48 epochs' seeds x 8 members, 1344 member pairs): max |dS| at
# ~1.2x the measurement; pooled Kendall tau >= 0.964 (round 4's bar, then on 12 seeds) = at most 24 discordant
# pairs; best / worst member may differ in at most 2 of the 48 epochs (round 4: 1 of 12).  Measured (round 5,
# profiles/r11c_rank_fidelity_ab.log + r11e_rank_fidelity_ab.log, four 12-seed sets): 18 pairs (8 + 4 + 4 + 2,
# tau 0.973), best 2 / worst 1 miss, max |dS| 0.0135 with forward_fp32's LoRA term on eggroll_lora_delta_f32;
# 16 pairs (5 + 3 + 6 + 2), best 2 / worst 2, max |dS| 0.0152 with the round-4 torch bmm form.  A 12-seed
# count moves by a few with any fp32-rounding-level change upstream, hence 48 seeds.
# The same bars at full model size: tests/test_gpu_parity_fullsize.py
RANK_BOUNDS = {"S_abs": 0.016, "pooled_tau": 0.964, "best_worst_misses": 2}


def kendall_tau(a, b):
    n = len(a)
    c = d = 0
    for i in range(n):
        for j in range(i + 1, n):
            s = np.sign(a[i] - a[j]) * np.sign(b[i] - b[j])
            c += s > 0
            d += s < 0
    return (c - d) / max(1, n * (n - 1) // 2)


def rel(a, b):
    return float((a.float() - b.float()).norm() / b.float().norm().clamp_min(1e-30))


@pytest.fixture(scope="module")
def stack(dev):
    cfg = SanaConfig(synthetic_weights=True, width_latent=4, height_latent=4, batches_per_gen=2, arch=TINY,
                     vae_widths=(16, 32, 32, 64, 64, 64), vae_layers=(1, 1, 1, 1, 1, 1))
    be = SanaBackend(str(dev), cfg)
    be.init_and_attach_lora()
    rewards = RewardModels.build(dev, tiny=True)
    return be, rewards, R.Rewards32(rewards)


@pytest.mark.parametrize("case", ["s0", "s1"])
def test_member_eval_bf16_vs_fp32_with_reference_noise(stack, dev, golden, case, monkeypatch):
    from hyperscalees_t2i_amd import lora
    # capture every linear's own output (the fused epilogues are bit-identical to this unfused form,
    # tests/test_gpu_engine.py::test_fused_epilogues_bit_identical)
    monkeypatch.setattr(lora, "FUSE_EPILOGUES", False)
    be, rewards, rewards32 = stack
    g = golden("g10_member_eval_injection.npz")
    params, shapes = be.collect_lora_params()
    assert [tuple(s) for s in shapes] == [tuple(s) for s in g["shapes"].tolist()]
    sigma = float(g[f"{case}/sigma"])
    pop = 8
    theta = flatten_params(params).to(dev)
    noiser = EggRollNoiser(shapes, sigma=sigma, lr_scale=0.1, rank=1, use_antithetic=True)
    fac = torch.from_numpy(noiser.layout.pack_factors(g[f"{case}/factors"])).to(dev)
    eps_ref = torch.from_numpy(g[f"{case}/eps"]).to(dev)
    tp = noiser.perturb(theta, fac, pop, 0, pop)
    assert torch.equal(tp, theta[None] + sigma * eps_ref)          # injected noise reproduced bit-exactly

    seed, gs = 5, 4.5
    info = be.step_sampling_info(seed)
    flat, m = info["flat_ids"], info["m"]
    B = len(flat)
    pe, am = be._gather(flat)

    # ---- build path (bf16, population-batched HIP kernels), LoRA outputs captured by hooks
    lin_out, tr_out = [], []
    hooks = [mod.register_forward_hook(lambda _m, _i, o: lin_out.append(o)) for mod in be.es_model.transformer.modules()
             if isinstance(mod, LoRALinear)]
    hooks.append(be.es_model.transformer.register_forward_hook(lambda _m, _i, o: tr_out.append(o)))
    try:
        imgs = be.generate_population(flat, seed, gs, tp)
    finally:
        for h in hooks:
            h.remove()
    j_of = torch.tensor([info["pid_to_j"][p] for p in flat], device=dev)
    feats = rewards.prompt_features(info["unique_texts"])
    rew = rewards.score(imgs, j_of.repeat(pop), feats)
    S, _ = aggregate_member_rewards(rew, flat, info["pid_to_j"], pop, m)
    fit = K.fitness(S, True)

    # ---- fp32 restatement, member by member (the reference loop)
    lat = be.es_model._latents(B, seed, 4, 4)
    feats32 = rewards32.prompt_features(info["unique_texts"])
    S32 = torch.empty((pop, m), device=dev)
    worst = {k: 0.0 for k in KEYS}
    worst["reward_model_abs"] = 0.0   # build reward towers on the fp32 image vs fp32 reward nets (diagnostic)
    # per-stage S breakdown: S rows when only one stage runs the build's precision
    S_tr = torch.empty((pop, m), device=dev)     # build transformer -> fp32 DC-AE -> fp32 towers
    S_img = torch.empty((pop, m), device=dev)    # build transformer + DC-AE (bf16 image) -> fp32 towers
    S_tow = torch.empty((pop, m), device=dev)    # fp32 image -> build towers
    S_tow16 = torch.empty((pop, m), device=dev)  # fp32 image -> plain-bf16 towers (round-2 towers)
    per_lin = {}
    lin_names = [n for n, mod in be.es_model.transformer.named_modules() if isinstance(mod, LoRALinear)]
    for k in range(pop):
        rec = []
        theta_k = theta + sigma * eps_ref[k]
        eps32, img32 = R.generate_fp32(be.es_model, theta_k, pe, am, lat, gs, rec)
        rw32 = rewards32.score(img32, j_of, feats32)
        rw_mix = rewards.score(img32.to(torch.bfloat16), j_of, feats)
        worst["reward_model_abs"] = max(worst["reward_model_abs"],
                                        float((rw_mix["combined"] - rw32["combined"]).abs().max()))
        agg = lambda rw: aggregate_member_rewards(rw, flat, info["pid_to_j"], 1, m)[0][0]  # noqa: E731
        S32[k] = agg(rw32)
        S_tow[k] = agg(rw_mix)
        img_t = R.decode_fp32(be.es_model, tr_out[0][k * B:(k + 1) * B], lat)
        S_tr[k] = agg(rewards32.score(img_t, j_of, feats32))
        S_img[k] = agg(rewards32.score(imgs[k * B:(k + 1) * B].float(), j_of, feats32))
        rewards.fp32_residual = False
        S_tow16[k] = agg(rewards.score(img32.to(torch.bfloat16), j_of, rewards.prompt_features(info["unique_texts"])))
        rewards.fp32_residual = True
        assert len(rec) == len(lin_out)
        for li, (a, b) in enumerate(zip(lin_out, rec)):
            a2 = a.reshape(-1, a.shape[-1])
            a2 = a2.view(pop, -1, a2.shape[-1])[k]
            b2 = b.reshape(-1, b.shape[-1])
            if a2.shape[0] * (B // m) == b2.shape[0]:
                # caption path (caption projection, attn2 to_k / to_v): the build evaluates the m distinct
                # prompts once per member; flat = repeat_batches(unique, R) puts them first, in order
                b2 = b2[: a2.shape[0]]
            e = rel(a2, b2)
            per_lin[li] = max(per_lin.get(li, 0.0), e)
            worst["lora_rel"] = max(worst["lora_rel"], e)
        worst["eps_rel"] = max(worst["eps_rel"], rel(tr_out[0][k * B:(k + 1) * B], eps32))
        worst["image_rel"] = max(worst["image_rel"], rel(imgs[k * B:(k + 1) * B], img32))
        worst["reward_abs"] = max(worst["reward_abs"],
                                  float((rew["combined"][k * B:(k + 1) * B] - rw32["combined"]).abs().max()))
    worst["S_abs"] = float((S - S32).abs().max())
    sc = fit["scores"].cpu().numpy()
    sc32, _, _ = O.ref_promptnorm(S32.cpu().numpy())
    spread = float(S32.std(0).mean())
    order, order32 = np.argsort(sc, kind="stable"), np.argsort(sc32, kind="stable")
    gaps = np.diff(np.sort(sc32))
    report = {"case": case, "sigma": sigma, **{k: round(v, 6) for k, v in worst.items()},
              "scores32": np.round(sc32, 5).tolist(), "scores": np.round(sc, 5).tolist(),
              "min_score_gap32": round(float(gaps.min()), 5),
              "S_member_spread": round(spread, 6), "rank_exact": bool(np.array_equal(order, order32)),
              "kendall_tau": round(float(kendall_tau(sc, sc32)), 4),
              "best_same": bool(order[-1] == order32[-1]), "worst_same": bool(order[0] == order32[0])}
    score_err = float(np.abs(sc - sc32).max())
    disc = [(i, j) for i in range(pop) for j in range(i + 1, pop)
            if np.sign(sc[i] - sc[j]) * np.sign(sc32[i] - sc32[j]) < 0]
    report["score_err"] = round(score_err, 5)
    report["discordant_gaps32"] = [round(float(abs(sc32[i] - sc32[j])), 5) for i, j in disc]
    stages = {}
    for name, Sx in (("transformer", S_tr), ("transformer+dcae", S_img), ("towers", S_tow),
                     ("towers_bf16_residual", S_tow16), ("all", S)):
        scx, _, _ = O.ref_promptnorm(Sx.cpu().numpy())
        stages[name] = {"S_abs": round(float((Sx - S32).abs().max()), 6), "kendall_tau": round(float(kendall_tau(scx, sc32)), 4)}
    report["stages"] = stages
    print("[fp32-parity]", json.dumps(report))
    print("[fp32-parity] per-linear rel", case, {lin_names[i] if i < len(lin_names) else i: round(v, 5)
                                                 for i, v in per_lin.items()})
    for k, b in BOUNDS[case].items():
        assert worst[k] <= b, (k, worst[k], b, report)
    if case == "s1":   # member signal >> bf16 noise: the reference's order up to near-ties
        assert score_err <= S1_SCORE_ERR and report["best_same"] and report["worst_same"], report
        assert all(gap <= 2 * score_err for gap in report["discordant_gaps32"]), report
    else:              # one seed's 8 members: a single swapped close pair reads 0.93 (pooled over seeds:
        assert report["kendall_tau"] >= 0.85, report   # test_rank_fidelity_over_seeds)


def test_rank_fidelity_over_seeds(stack, dev, golden):
    """Fitness-order agreement with the fp32 restatement at the BASELINE sigma (1e-2), product path
    (fused epilogues, shared projections), over several epochs' seeds (latents + prompt draw differ):
    one 8-member tau is a coarse statistic (one swapped pair = 0.93), so the bar is on the pooled
    discordant-pair fraction and on best / worst member agreement.  Reference noise injected (g10).
    The per-stage breakdown is pooled over the same 12 seeds: S recomputed with only one stage at the
    build's precision (transformer -> fp32 DC-AE -> fp32 towers; transformer + DC-AE image -> fp32
    towers; fp32 image -> build towers), so the discordant pairs are attributed to a stage."""
    be, rewards, rewards32 = stack
    g = golden("g10_member_eval_injection.npz")
    params, shapes = be.collect_lora_params()
    sigma, pop = float(g["s0/sigma"]), 8
    theta = flatten_params(params).to(dev)
    noiser = EggRollNoiser(shapes, sigma=sigma, lr_scale=0.1, rank=1, use_antithetic=True)
    fac = torch.from_numpy(noiser.layout.pack_factors(g["s0/factors"])).to(dev)
    eps_ref = torch.from_numpy(g["s0/eps"]).to(dev)
    tp = noiser.perturb(theta, fac, pop, 0, pop)
    stages = ("all", "transformer", "transformer+dcae", "towers")
    st = {k: {"disc": 0, "best": 0, "worst": 0, "S_abs": 0.0} for k in stages}
    taus, pairs, spread = [], 0, []
    # 48 epochs' seeds, 1344 member pairs (one pair = 0.0015 of pooled tau); EGG_RANK_SEEDS=lo:hi re-draws them (A/B)
    seeds = tuple(range(*map(int, os.environ.get("EGG_RANK_SEEDS", "5:53").split(":"))))
    for seed in seeds:
        info = be.step_sampling_info(seed)
        flat, m = info["flat_ids"], info["m"]
        B = len(flat)
        pe, am = be._gather(flat)
        tr_out = []
        hook = be.es_model.transformer.register_forward_hook(lambda _m, _i, o: tr_out.append(o))
        try:
            imgs = be.generate_population(flat, seed, 4.5, tp)
        finally:
            hook.remove()
        j_of = torch.tensor([info["pid_to_j"][p] for p in flat], device=dev)
        feats = rewards.prompt_features(info["unique_texts"])
        rew = rewards.score(imgs, j_of.repeat(pop), feats)
        Sx = {"all": aggregate_member_rewards(rew, flat, info["pid_to_j"], pop, m)[0]}
        lat = be.es_model._latents(B, seed, 4, 4)
        feats32 = rewards32.prompt_features(info["unique_texts"])
        agg = lambda rw: aggregate_member_rewards(rw, flat, info["pid_to_j"], 1, m)[0][0]  # noqa: E731
        rows = {k: [] for k in ("S32", "transformer", "transformer+dcae", "towers")}
        for k in range(pop):
            img32 = R.generate_fp32(be.es_model, theta + sigma * eps_ref[k], pe, am, lat, 4.5)[1]
            rows["S32"].append(agg(rewards32.score(img32, j_of, feats32)))
            rows["transformer"].append(agg(rewards32.score(R.decode_fp32(be.es_model, tr_out[0][k * B:(k + 1) * B], lat),
                                                           j_of, feats32)))
            rows["transformer+dcae"].append(agg(rewards32.score(imgs[k * B:(k + 1) * B].float(), j_of, feats32)))
            rows["towers"].append(agg(rewards.score(img32.to(torch.bfloat16), j_of, feats)))
        S32 = torch.stack(rows["S32"])
        for k in ("transformer", "transformer+dcae", "towers"):
            Sx[k] = torch.stack(rows[k])
        sc32, _, _ = O.ref_promptnorm(S32.cpu().numpy())
        o32 = np.argsort(sc32, kind="stable")
        for name in stages:
            sc = (K.fitness(Sx[name], True)["scores"].cpu().numpy() if name == "all"
                  else O.ref_promptnorm(Sx[name].cpu().numpy())[0])
            t = kendall_tau(sc, sc32)
            if name == "all":
                taus.append(round(float(t), 4))
            o = np.argsort(sc, kind="stable")
            d = st[name]
            d["disc"] += round((1 - t) / 2 * (pop * (pop - 1) // 2))
            d["best"] += int(o[-1] == o32[-1])
            d["worst"] += int(o[0] == o32[0])
            d["S_abs"] = max(d["S_abs"], float((Sx[name] - S32).abs().max()))
        pairs += pop * (pop - 1) // 2
        spread.append(float(S32.std(0).mean()))
    for d in st.values():
        d["pooled_tau"] = round(1 - 2 * d["disc"] / pairs, 4)
        d["S_abs"] = round(d["S_abs"], 6)
    a = st["all"]
    report = {"sigma": sigma, "seeds": list(seeds), "kendall_tau": taus, "pooled_tau": a["pooled_tau"],
              "discordant_pairs": a["disc"], "pairs": pairs, "best_same": a["best"], "worst_same": a["worst"],
              "S_abs_max": a["S_abs"], "S_member_spread_mean": round(float(np.mean(spread)), 6),
              "stages": {k: st[k] for k in stages if k != "all"}}
    print("[fp32-parity] rank fidelity over seeds", json.dumps(report))
    assert a["S_abs"] <= RANK_BOUNDS["S_abs"], report
    assert report["pooled_tau"] >= RANK_BOUNDS["pooled_tau"], report
    assert a["best"] >= len(seeds) - RANK_BOUNDS["best_worst_misses"], report
    assert a["worst"] >= len(seeds) - RANK_BOUNDS["best_worst_misses"], report
