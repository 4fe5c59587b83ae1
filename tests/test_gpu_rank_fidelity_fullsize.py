"""Fitness-rank fidelity at the BASELINE model size (Sana-Sprint 1.6B, 1024 px, CLIP-H/14 PickScore +
CLIP-B/32) over 12 epochs' seeds: the bf16 product path vs the fp32 restatement
(oracle/member_eval_fp32.py) on the same eps, pop 8, egg rank 1, sigma 1e-2.

The reference scores every member of an epoch independently (unifed_es.py:159-215) and ranks the
promptnorm fitness (utills.py:310-330, models/SanaSprint.py:122-160 for the member forward); the build's
fitness order must follow the fp32 order up to members that are tied within its own score error.

Each seed is its own test (progress is visible per epoch); the fp32 side is computed once per seed
and the bf16 side twice — through the product's cross-attention (the two-half online softmax,
eggroll_cross_attention_sel variant 0) and through the two-pass form (variant 1) — so the per-epoch
max |score - score32| of the two forms is measured on the same epochs.  The last
test pools the 12 x 28 = 336 member pairs and asserts the bar:

  * pooled Kendall tau >= 0.964 (the tiny-architecture bar, tests/test_gpu_parity_fp32.py);
  * every discordant pair and best / worst miss is a near-tie: its fp32 score gap at most 1.5x that
    epoch's largest |score - score32|;
  * max |S - S32| <= 3e-3 (DESIGN.md §3.2 "full size").
"""
import json
import os
from pathlib import Path
from types import SimpleNamespace

import numpy as np
import pytest
import torch

from hyperscalees_t2i_amd import kernels as K
from hyperscalees_t2i_amd.es import EggRollNoiser
from hyperscalees_t2i_amd.es_step import aggregate_member_rewards
from oracle import eggroll_oracle as O
from oracle import member_eval_fp32 as R

pytestmark = pytest.mark.gpu

RANK_BOUNDS = {"S_abs": 3e-3, "pooled_tau": 0.964, "near_tie": 1.5}
SEEDS = tuple(range(5, 17))
VARIANTS = {"online": 0, "two_pass": 1}     # eggroll_cross_attention_sel: 0 = the product's automatic choice
DECODE_CHUNK = 4
POP, SIGMA = 8, 1e-2
_RESULTS = {}


def kendall_tau(a, b):
    n = len(a)
    c = d = 0
    for i in range(n):
        for j in range(i + 1, n):
            s = np.sign(a[i] - a[j]) * np.sign(b[i] - b[j])
            c += s > 0
            d += s < 0
    return (c - d) / max(1, n * (n - 1) // 2)


@pytest.fixture(scope="module")
def full(dev):
    import bench
    torch.backends.cudnn.benchmark = False
    args = SimpleNamespace(workload="sana", small=False, pop_per_gpu=POP, latent=32)
    backend, engine, noiser, theta, _ = bench.build(args, 1, 0, dev)
    rewards = engine.rewards
    yield backend, rewards, R.Rewards32(rewards), theta


@pytest.fixture
def fp32_math():
    old = torch.backends.cuda.matmul.allow_tf32, torch.backends.cudnn.allow_tf32
    torch.backends.cuda.matmul.allow_tf32 = torch.backends.cudnn.allow_tf32 = False
    yield
    torch.backends.cuda.matmul.allow_tf32, torch.backends.cudnn.allow_tf32 = old


def _epoch_stats(sc, sc32):
    """Kendall tau, discordant pairs, best / worst hits and the near-tie ratio of one epoch."""
    pop = len(sc)
    t = kendall_tau(sc, sc32)
    o, o32 = np.argsort(sc, kind="stable"), np.argsort(sc32, kind="stable")
    err = float(np.abs(sc - sc32).max())
    gaps = [abs(sc32[i] - sc32[j]) for i in range(pop) for j in range(i + 1, pop)
            if np.sign(sc[i] - sc[j]) * np.sign(sc32[i] - sc32[j]) < 0]
    gaps += [sc32[o32[-1]] - sc32[o[-1]], sc32[o[0]] - sc32[o32[0]]]   # best / worst misses (0 if none)
    return {"tau": round(float(t), 4), "disc": int(round((1 - t) / 2 * (pop * (pop - 1) // 2))),
            "best": int(o[-1] == o32[-1]), "worst": int(o[0] == o32[0]), "score_err": err,
            "tie_ratio": float(max(gaps)) / max(err, 1e-12)}


@pytest.mark.timeout(600)
@pytest.mark.parametrize("seed", SEEDS)
def test_rank_fidelity_epoch(full, dev, fp32_math, monkeypatch, seed):
    be, rewards, rewards32, theta = full
    params, shapes = be.collect_lora_params()
    gs = be.cfg.guidance_scale
    noiser = EggRollNoiser(shapes, sigma=SIGMA, lr_scale=0.1, rank=1, use_antithetic=True)
    fac = noiser.sample_factors(POP, dev, seed=seed)
    eps = noiser.eps_from_factors(fac, POP)
    tp = noiser.perturb(theta, fac, POP, 0, POP)
    info = be.step_sampling_info(seed)
    flat, m = info["flat_ids"], info["m"]
    B = len(flat)
    j_of = torch.tensor([info["pid_to_j"][p] for p in flat], device=dev)
    feats = rewards.prompt_features(info["unique_texts"])
    S = {}
    for name, var in VARIANTS.items():
        monkeypatch.setattr(K, "XATTN_VARIANT", var)
        imgs = be.generate_population(flat, seed, gs, tp)
        S[name] = aggregate_member_rewards(rewards.score(imgs, j_of.repeat(POP), feats), flat, info["pid_to_j"],
                                           POP, m)[0]
        del imgs
    monkeypatch.setattr(K, "XATTN_VARIANT", 0)
    pe, am = be._gather(flat)
    lat = be.es_model._latents(B, seed, be.cfg.height_latent, be.cfg.width_latent)
    feats32 = rewards32.prompt_features(info["unique_texts"])
    rows = []
    for k in range(POP):
        with torch.no_grad():
            img32 = R.generate_fp32(be.es_model, theta + SIGMA * eps[k], pe, am, lat, gs, decode_chunk=DECODE_CHUNK)[1]
            rows.append(aggregate_member_rewards(rewards32.score(img32, j_of, feats32), flat, info["pid_to_j"], 1, m)[0][0])
        del img32
    S32 = torch.stack(rows)
    sc32, _, _ = O.ref_promptnorm(S32.cpu().numpy())
    rec = {"S_member_spread": float(S32.std(0).mean())}
    for name in VARIANTS:
        sc = K.fitness(S[name], True)["scores"].cpu().numpy()
        st = _epoch_stats(sc, sc32)
        st["S_abs"] = float((S[name] - S32).abs().max())
        rec[name] = st
    _RESULTS[seed] = rec
    print(f"[rank-fidelity-full] seed {seed}", json.dumps(rec))


def test_rank_fidelity_pooled():
    missing = [s for s in SEEDS if s not in _RESULTS]
    if missing:
        pytest.skip(f"per-seed epochs did not all run (missing {missing})")
    pairs = len(SEEDS) * POP * (POP - 1) // 2
    report = {"sigma": SIGMA, "pop": POP, "seeds": list(SEEDS), "pairs": pairs,
              "S_member_spread_mean": round(float(np.mean([_RESULTS[s]["S_member_spread"] for s in SEEDS])), 6)}
    for name in VARIANTS:
        ep = [_RESULTS[s][name] for s in SEEDS]
        disc = sum(e["disc"] for e in ep)
        report[name] = {"pooled_tau": round(1 - 2 * disc / pairs, 4), "discordant_pairs": disc,
                        "kendall_tau": [e["tau"] for e in ep],
                        "best_same": sum(e["best"] for e in ep), "worst_same": sum(e["worst"] for e in ep),
                        "score_err_per_epoch": [round(e["score_err"], 5) for e in ep],
                        "score_err_max": round(max(e["score_err"] for e in ep), 5),
                        "score_err_mean": round(float(np.mean([e["score_err"] for e in ep])), 5),
                        "S_abs_max": round(max(e["S_abs"] for e in ep), 6),
                        "misorder_gap_over_score_err": round(max(e["tie_ratio"] for e in ep), 4)}
    print("[rank-fidelity-full] pooled", json.dumps(report))
    out = Path(os.environ.get("GRAFT_REPO_ROOT", Path(__file__).resolve().parent.parent)) / "gpurun_out"
    try:
        out.mkdir(exist_ok=True)
        (out / "rank_fidelity_fullsize.json").write_text(json.dumps(report, indent=1))
    except OSError:
        pass
    prod = report["online"]
    assert prod["S_abs_max"] <= RANK_BOUNDS["S_abs"], report
    assert prod["pooled_tau"] >= RANK_BOUNDS["pooled_tau"], report
    assert prod["misorder_gap_over_score_err"] <= RANK_BOUNDS["near_tie"], report
