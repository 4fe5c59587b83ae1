"""VAR model-level parity (BASELINE configs[0]: VAR-d16 class-conditional, LoRA r 4, pop 4) against
the reference's own VAR_models, via tests/golden/g11_var_model.npz (make_golden.gen_var_model: the
reference run on CPU fp32 at depth 2 / VQVAE ch 32 with deterministic synthetic weights and the
PEFT LoRA formula hooked onto every target).

CPU (`-m "not gpu"`):
  * the module trees carry the reference's parameter names and shapes (state-dict drop-in) and the
    LoRA theta layout equals the reference's (suffix-matched targets, module order);
  * the restated top-k / top-p sampler replays the reference's CPU draws bit-exactly (scales 0-3,
    exact fp32 CFG logits, Generator seeded with g_seed as var.py:143-144 does).
GPU (`-m gpu`):
  * teacher-forced on the reference's token maps, every scale's CFG logits, f_hat and the decoded
    image agree with the reference within the stated bf16 tolerances;
  * the population path (3 members, one forward) reproduces the single-member path per member;
  * a free-running population generation is deterministic and a whole ES epoch on the VAR backend
    matches the oracle's update of the same S.
"""
import numpy as np
import pytest
import torch

from hyperscalees_t2i_amd.sana import attach_lora
from hyperscalees_t2i_amd.var import (VARArch, VARClassGenerator, VARTransformer, VQVAEDecode,
                                      sample_with_top_k_top_p_)
from tests.var_weights import TARGETS, TINY, synth_state

ARCH = VARArch(depth=TINY["depth"], vae_ch=TINY["vae_ch"])

# Stated tolerances, bf16 transformer / decoder vs the reference's fp32 (measured values: DESIGN §3.3).
# Measured on MI355X (round 2): worst logit rel 0.0217, image max 0.041, mean 0.0039; bounds ~2x.
LOGIT_REL = 0.04      # ||dlogits|| / ||logits|| per scale (teacher-forced)
FHAT_ABS = 1e-4       # f_hat: fp32 codebook / resampling / Phi path on identical tokens
IMAGE_ABS = 0.08      # decoded image in [0, 1], max |d| (bf16 convolutions; ~20/255)
IMAGE_MEAN = 8e-3     # mean |d| (~2/255)
POP_REL = 3e-2        # population (fused LoRA epilogue) vs single-member (bf16 y + separate LoRA add) logits


def _keys(mod):
    return [f"{n}:{'x'.join(map(str, p.shape))}" for n, p in mod.named_parameters()]


def test_var_state_dict_names_match_reference(golden):
    d = golden("g11_var_model.npz")
    with torch.device("meta"):
        var, vae = VARTransformer(ARCH), VQVAEDecode(ARCH)
    assert _keys(var) == str(d["var_keys"]).split("\x1f")
    assert sorted(_keys(vae)) == sorted(str(d["dec_keys"]).split("\x1f"))
    attach_lora(var, TINY["lora_r"], TINY["lora_alpha"], TARGETS)
    shapes = [tuple(p.shape) for p in var.parameters() if p.requires_grad]
    assert shapes == [tuple(s) for s in d["lora_shapes"]]
    assert sum(a * b for a, b in shapes) == d["theta"].size


def test_var_sampler_replays_reference_draws(golden):
    """helpers.py:6-19 restated: same masks, same softmax, same multinomial stream."""
    d = golden("g11_var_model.npz")
    cfg, top_k, top_p, g_seed = d["meta"]
    rng = torch.Generator().manual_seed(int(g_seed))
    for si in range(4):
        logits = torch.from_numpy(d[f"logit_full{si}"].copy())
        idx = sample_with_top_k_top_p_(logits, top_k=int(top_k), top_p=float(top_p), rng=rng, num_samples=1)[:, :, 0]
        assert torch.equal(idx, torch.from_numpy(d[f"idx{si}"].astype(np.int64))), si


# ---------------------------------------------------------------------------------------------------
# GPU
# ---------------------------------------------------------------------------------------------------


def _build(dev, theta_np):
    gen = VARClassGenerator(device=str(dev), arch=ARCH)
    gen.load_reference_state(synth_state([(n, tuple(p.shape)) for n, p in gen.var.named_parameters()]),
                             synth_state([(n, tuple(p.shape)) for n, p in gen.vae.named_parameters()]))
    attach_lora(gen.var, TINY["lora_r"], TINY["lora_alpha"], TARGETS)
    theta = torch.from_numpy(theta_np.copy()).to(dev)
    off = 0
    with torch.no_grad():
        for p in gen.var.parameters():
            if p.requires_grad:
                p.copy_(theta[off:off + p.numel()].view_as(p))
                off += p.numel()
    assert off == theta.numel()
    return gen, theta


def _forced(d, n, dev):
    return [torch.from_numpy(d[f"idx{si}"].astype(np.int64)).to(dev).repeat(n, 1) for si in range(len(ARCH.patch_nums))]


@pytest.mark.gpu
def test_var_teacher_forced_matches_reference(golden, dev):
    d = golden("g11_var_model.npz")
    cfg, top_k, top_p, g_seed = d["meta"]
    gen, _ = _build(dev, d["theta"])
    labels = torch.from_numpy(d["labels"]).to(dev)
    f_hat, idx, logits = gen.infer.run(labels, 1, int(g_seed), float(cfg), int(top_k), float(top_p),
                                       force_idx=_forced(d, 1, dev), keep_logits=True)
    worst = 0.0
    for si in range(len(ARCH.patch_nums)):
        pos = torch.from_numpy(d[f"pos{si}"]).to(dev)
        mine = logits[si][0][:, pos]                                         # [B, |pos|, V]
        ref = torch.from_numpy(d[f"logit_sub{si}"].astype(np.float32)).to(dev)
        rel = float((mine - ref).norm() / ref.norm())
        worst = max(worst, rel)
        assert rel < LOGIT_REL, (si, rel)
        if si <= 3:
            full = torch.from_numpy(d[f"logit_full{si}"]).to(dev)
            assert float((logits[si][0] - full).norm() / full.norm()) < LOGIT_REL, si
    fh = torch.from_numpy(d["f_hat"]).to(dev)
    assert float((f_hat - fh).abs().max()) < FHAT_ABS
    img = (gen.vae.fhat_to_img(f_hat).float() + 1) * 0.5
    ref_img = torch.from_numpy(d["image"].astype(np.float32)).to(dev)
    err = (img.clamp(0, 1) - ref_img).abs()
    print(f"[var parity] worst logit rel {worst:.4f}  image max {float(err.max()):.4f} mean {float(err.mean()):.5f}")
    assert float(err.max()) < IMAGE_ABS and float(err.mean()) < IMAGE_MEAN


@pytest.mark.gpu
def test_var_population_matches_single_member(golden, dev):
    """One forward for 3 members (theta_pop rows) == three single-member forwards (teacher forced)."""
    d = golden("g11_var_model.npz")
    cfg, top_k, top_p, g_seed = d["meta"]
    gen, theta = _build(dev, d["theta"])
    g = torch.Generator(device=dev).manual_seed(3)
    pop = torch.stack([theta + 0.02 * torch.randn(theta.shape, generator=g, device=dev) for _ in range(3)])
    labels = torch.from_numpy(d["labels"]).to(dev)
    gen.ctx.theta_pop, gen.ctx.n_members = pop, 3
    from hyperscalees_t2i_amd.lora import set_population
    set_population(gen.var, gen.ctx)
    try:
        f_pop, _, lg_pop = gen.infer.run(labels, 3, int(g_seed), float(cfg), int(top_k), float(top_p),
                                         force_idx=_forced(d, 3, dev), keep_logits=True)
    finally:
        set_population(gen.var, None)
        gen.ctx.theta_pop = None
    B = labels.numel()
    for k in range(3):
        with torch.no_grad():
            off = 0
            for p in gen.var.parameters():
                if p.requires_grad:
                    p.copy_(pop[k, off:off + p.numel()].view_as(p))
                    off += p.numel()
        f1, _, lg1 = gen.infer.run(labels, 1, int(g_seed), float(cfg), int(top_k), float(top_p),
                                   force_idx=_forced(d, 1, dev), keep_logits=True)
        for si in range(len(ARCH.patch_nums)):
            a, b = lg_pop[si][k], lg1[si][0]
            assert float((a - b).norm() / b.norm()) < POP_REL, (k, si)
        assert torch.allclose(f_pop[k * B:(k + 1) * B], f1, atol=1e-5)


@pytest.mark.gpu
def test_var_free_generation_deterministic(golden, dev):
    d = golden("g11_var_model.npz")
    gen, theta = _build(dev, d["theta"])
    pop = theta[None].repeat(2, 1).contiguous()
    labels = torch.tensor([3, 980, 3, 980], device=dev)
    a = gen.generate_population(labels, pop, seed=7, guidance_scale=4.0)
    b = gen.generate_population(labels, pop, seed=7, guidance_scale=4.0)
    assert a.shape == (8, 3, 256, 256) and torch.isfinite(a).all()
    assert torch.equal(a, b)
    # identical members + identical seeds -> identical images (member streams are independent copies)
    assert torch.equal(a[:4], a[4:])
    imgs, _ = gen.generate(seed=7, guidance_scale=4.0, class_ids=[[3, 980], [3, 980]], return_grouped=True)
    assert len(imgs) == 2 and len(imgs[0]) == 2 and imgs[0][0].size == (256, 256)


@pytest.mark.gpu
def test_var_es_epoch_matches_oracle(dev):
    """BASELINE configs[0] shape (pop 4, antithetic, 2 classes x 2 batches) through ESEngine on the
    tiny VAR: theta' == the oracle's restatement of unifed_es.py:227-281 on the engine's own S."""
    from hyperscalees_t2i_amd.backend import VarBackend, VarConfig
    from hyperscalees_t2i_amd.es import EggRollNoiser, flatten_params
    from hyperscalees_t2i_amd.es_step import ESConfig, ESEngine
    from hyperscalees_t2i_amd.rewards import RewardModels
    from oracle import eggroll_oracle as O
    be = VarBackend(str(dev), VarConfig(arch=ARCH, classes_per_gen=2, batches_per_gen=2, ckpt_dir="/nonexistent", synthetic_if_missing=True))
    be.init_and_attach_lora()
    params, shapes = be.collect_lora_params()
    theta = flatten_params(params).to(dev)
    noiser = EggRollNoiser(shapes, sigma=1e-2, lr_scale=1e-1, rank=1, use_antithetic=True)
    eng = ESEngine(be, RewardModels.build(dev, tiny=True), noiser, ESConfig(pop_size=4, theta_max_norm=40.0), dev)
    new, stats = eng.step(theta, seed=3, guidance_scale=4.0)
    torch.cuda.synchronize()
    S = stats["_S"].numpy()
    assert S.shape == (4, 2) and np.isfinite(S).all()
    eps = noiser.eps_from_factors(noiser.sample_factors(4, dev, seed=3), 4).cpu().numpy()
    ref, _ = O.ref_es_tail(S, eps, theta.cpu().numpy(), promptnorm=True, lr_scale=1e-1, sigma=1e-2,
                           max_step_norm=0.0, theta_max_norm=40.0)
    assert np.abs(new.cpu().numpy() - ref).max() < 1e-5
