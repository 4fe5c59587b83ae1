"""Infinity host (BASELINE configs[4]) on the GPU, tiny architecture: the population pass vs the fp32
restatement of the same architecture with member factors from theta_k (oracle/infinity_fp32.py) and
vs one member at a time, both teacher-forced (the same bits at every scale); sampled generation
(shapes, member differences, the reference's micro-batch generator semantics); a full ES epoch vs the
oracle's epoch tail.  The architecture restates the Infinity repo (absent here): parity UNPINNED."""
import numpy as np
import pytest
import torch

from hyperscalees_t2i_amd.backend import InfinityBackend, InfinityConfig
from hyperscalees_t2i_amd.es import EggRollNoiser, flatten_params, unflatten_to_params
from hyperscalees_t2i_amd.es_step import ESConfig, ESEngine
from hyperscalees_t2i_amd.infinity import InfinityArch
from hyperscalees_t2i_amd.rewards import RewardModels
from oracle import eggroll_oracle as O

pytestmark = pytest.mark.gpu

TINY = InfinityArch(depth=2, embed_dim=256, num_heads=2, block_chunks=2, text_channels=256, codebook_dim=4,
                    spatial_patchify=1, vae_widths=(32, 32, 64, 64))


@pytest.fixture(scope="module")
def setup(dev):
    cfg = InfinityConfig(synthetic_weights=True, arch=TINY, pn="0.06M", batches_per_gen=2, micro_batch=0,
                         synthetic_prompt_lens=(5, 40), vae_chunk=8)
    be = InfinityBackend(str(dev), cfg)
    be.init_and_attach_lora()
    params, shapes = be.collect_lora_params()
    return be, params, shapes


def _forced(be, flat, n, seed=0):
    g = torch.Generator().manual_seed(seed)
    a = be.es_model.arch
    return [torch.randint(0, 2, (n * len(flat), h * w, a.d_tok), generator=g) for _, h, w in be.es_model.scale_schedule]


def _pop_logits(be, flat, tp, bits):
    uniq = list(dict.fromkeys(flat))
    idx = torch.tensor([uniq.index(f) for f in flat])
    c = be.cfg
    imgs = be.es_model.generate_population([be._dev_kv[p] for p in uniq], [be.lens_list[p] for p in uniq], idx, tp, 1,
                                           c.cfg_list, c.tau_list, c.top_k, c.top_p, 0, force_bits=bits,
                                           keep_logits=True)
    return imgs, be.es_model.last_logits, uniq, idx


def test_lora_layout(setup):
    be, params, shapes = setup
    assert [tuple(s) for s in shapes] == [(2, 256), (1024, 2)] * 2


def test_population_vs_fp32_restatement_teacher_forced(setup, dev):
    """Member k's per-scale CFG logits (same forced bits) vs the fp32 restatement: relative error per
    scale.  sigma 5e-2 so the members' LoRA terms are well above bf16 noise; the two members differ."""
    from oracle import infinity_fp32 as Z
    be, params, shapes = setup
    theta0 = flatten_params(params).to(dev)
    noiser = EggRollNoiser(shapes, sigma=5e-2, lr_scale=0.1, rank=1, use_antithetic=True)
    pop = 2
    tp = noiser.perturb(theta0, noiser.sample_factors(pop, dev, seed=4), pop, 0, pop)
    flat = be.step_sampling_info(1)["flat_ids"]
    bits = _forced(be, flat, pop)
    imgs, logits, uniq, idx = _pop_logits(be, flat, tp, bits)
    B = len(flat)
    assert imgs.shape == (pop * B, 3, 256, 256) and torch.isfinite(imgs).all()
    sched = be.es_model.scale_schedule
    T = len(sched)
    worst = 0.0
    for k in range(pop):
        ref = Z.member_logits_fp32(be.es_model.transformer, [be._dev_kv[p] for p in uniq],
                                   [be.lens_list[p] for p in uniq], idx, tp[k], sched, [3.0] * T, [1.0] * T,
                                   [b.view(pop, B, *b.shape[1:])[k] for b in bits])
        for si in range(T):
            got = logits[si].view(pop, B, -1, 2)[k]
            worst = max(worst, ((got - ref[si]).norm() / ref[si].norm()).item())
    print("[infinity-fp32] worst per-scale logit rel err", worst)
    assert worst < 3e-2, worst
    d = (logits[-1].view(pop, B, -1, 2)[0] - logits[-1].view(pop, B, -1, 2)[1]).abs().max().item()
    assert d > 0


def test_population_vs_single_member_teacher_forced(setup, dev):
    be, params, shapes = setup
    theta0 = flatten_params(params).to(dev)
    noiser = EggRollNoiser(shapes, sigma=5e-2, lr_scale=0.1, rank=1, use_antithetic=True)
    pop = 3
    tp = noiser.perturb(theta0, noiser.sample_factors(pop, dev, seed=6), pop, 0, pop)
    flat = be.step_sampling_info(2)["flat_ids"]
    bits = _forced(be, flat, pop, seed=1)
    _, logits, uniq, idx = _pop_logits(be, flat, tp, bits)
    B = len(flat)
    es = be.es_model
    c = be.cfg
    for k in range(pop):
        unflatten_to_params(tp[k], params, shapes)
        es._generate([be._dev_kv[p] for p in uniq], [be.lens_list[p] for p in uniq], idx.to(dev), 1, 1, c.cfg_list,
                     c.tau_list, c.top_k, c.top_p, 0, None, force_bits=[b.view(pop, B, *b.shape[1:])[k] for b in bits],
                     keep_logits=True)
        for si, one in enumerate(es.last_logits):
            got = logits[si].view(pop, B, -1, 2)[k]
            rel = ((got - one.view(B, -1, 2)).norm() / one.norm()).item()
            assert rel < 2e-2, (k, si, rel)
    unflatten_to_params(theta0, params, shapes)


def test_sampled_generation_and_micro_batch_semantics(setup, dev):
    """Sampled bits: members differ; with micro_batch 2 every chunk restarts the generator at `seed`,
    so the first chunk's bits equal those of a 2-image call on its own (up to bf16 ties: >= 99 %)."""
    be, params, shapes = setup
    es, c = be.es_model, be.cfg
    flat = be.step_sampling_info(3)["flat_ids"]
    theta0 = flatten_params(params).to(dev)
    noiser = EggRollNoiser(shapes, sigma=5e-2, lr_scale=0.1, rank=1, use_antithetic=True)
    tp = noiser.perturb(theta0, noiser.sample_factors(2, dev, seed=2), 2, 0, 2)
    uniq = list(dict.fromkeys(flat))
    idx = torch.tensor([uniq.index(f) for f in flat])
    kv, lens = [be._dev_kv[p] for p in uniq], [be.lens_list[p] for p in uniq]
    imgs = es.generate_population(kv, lens, idx, tp, 5, c.cfg_list, c.tau_list, c.top_k, c.top_p, micro_batch=2)
    B = len(flat)
    assert imgs.shape == (2 * B, 3, 256, 256) and torch.isfinite(imgs).all()
    bits_mb = [b.view(2, B, -1) for b in es.last_bits]
    assert any((b[0] != b[1]).any() for b in bits_mb)
    es.generate_population(kv, lens, idx[:2], tp, 5, c.cfg_list, c.tau_list, c.top_k, c.top_p, micro_batch=0)
    agree = np.mean([(b2.view(2, 2, -1) == b[:, :2]).float().mean().item() for b2, b in zip(es.last_bits, bits_mb)])
    assert agree >= 0.99, agree


def test_engine_step_matches_oracle(setup, dev):
    be, params, shapes = setup
    rewards = RewardModels.build(dev, tiny=True, synthetic=True)
    theta = flatten_params(params).to(dev)
    pop = 4
    noiser = EggRollNoiser(shapes, sigma=1e-2, lr_scale=1e-1, rank=1, use_antithetic=True)
    eng = ESEngine(be, rewards, noiser, ESConfig(pop_size=pop, egg_rank=1, promptnorm=True, theta_max_norm=40.0), dev)
    new, st = eng.step(theta, seed=3, guidance_scale=be.cfg.guidance_scale)
    eps = noiser.eps_from_factors(noiser.sample_factors(pop, dev, seed=3), pop).cpu().numpy()
    ref, info = O.ref_es_tail(st["_S"].numpy(), eps, theta.cpu().numpy(), promptnorm=True, lr_scale=1e-1,
                              sigma=1e-2, max_step_norm=0.0, theta_max_norm=40.0)
    np.testing.assert_allclose(new.cpu().numpy(), ref, rtol=1e-5, atol=1e-8)
    assert np.array_equal(st["_fitness"]["order"].numpy(), info["order"])
    assert np.isfinite(st["summary/mean_reward"])


def test_generate_flat_returns_pil(setup):
    be, _, _ = setup
    be.cfg.micro_batch = 2
    try:
        imgs = be.generate_flat([0, 1, 0], seed=0, guidance_scale=3.0)
    finally:
        be.cfg.micro_batch = 0
    assert len(imgs) == 3 and imgs[0].size == (256, 256) and imgs[0].mode == "RGB"


def test_qk_norm_rope_kv_cache_append(dev):
    """eggroll_qk_norm_rope_kv: q normalised + rotated + per-head scaled in place, k written into a cache
    slice at [seq, row0 + t] with the values copied alongside == the torch form (within one bf16 rounding;
    the cache outside the slice untouched)."""
    from hyperscalees_t2i_amd import kernels as K
    from hyperscalees_t2i_amd.infinity import _rms_rope_torch
    g = torch.Generator(device=dev).manual_seed(3)
    S, l, H, C, ltot, row0 = 3, 20, 2, 256, 57, 11
    qkv = torch.randn(S * l, 3 * C, generator=g, device=dev).bfloat16()
    ang = torch.rand(l, 64, generator=g, device=dev) * 6.3
    cos, sin = torch.cos(ang).contiguous(), torch.sin(ang).contiguous()
    hs = (torch.rand(H, generator=g, device=dev) + 0.5).bfloat16().float()
    ones = torch.ones(128, device=dev, dtype=torch.bfloat16)
    cache = torch.randn(2, S, ltot, C, generator=g, device=dev).bfloat16()
    ref_q = qkv[:, :C].clone()
    _rms_rope_torch(ref_q, H, 128, 1e-12, cos, sin)
    ref_q = (ref_q.view(-1, H, 128) * hs.bfloat16().view(1, H, 1)).view(-1, C)
    ref_k = qkv[:, C:2 * C].clone()
    _rms_rope_torch(ref_k, H, 128, 1e-12, cos, sin)
    ref_cache = cache.clone()
    ref_cache[0, :, row0:row0 + l] = ref_k.view(S, l, C)
    ref_cache[1, :, row0:row0 + l] = qkv[:, 2 * C:].view(S, l, C)
    x = qkv.clone()
    K.qk_norm_rope_kv(x[:, :C], ones, 1e-12, cos, sin, H, hscale=hs)
    K.qk_norm_rope_kv(x[:, C:2 * C], ones, 1e-12, cos, sin, H, out=cache[0], rows_per_seq=l, row0=row0,
                      vin=x[:, 2 * C:], vout=cache[1])
    tol = lambda a, b: ((a.float() - b.float()).abs() <= b.float().abs() * 2 ** -7 + 1e-6).all()  # noqa: E731
    assert tol(x[:, :C], ref_q)
    assert tol(cache, ref_cache)
    assert torch.equal(cache[:, :, :row0], ref_cache[:, :, :row0]) and torch.equal(cache[1], ref_cache[1])


def test_loaded_infinity_generates_identically(setup, dev, tmp_path):
    """The synthetic model exported in the Infinity repo's layout (checkpoints.save_infinity_checkpoint: a shard
    directory + the BSQ-VAE .pth) and loaded back through InfinityConfig(model_path=..., checkpoint_type=
    "torch_shard", vae_path=...) gives bit-identical sampled bits and images for a population pass."""
    from hyperscalees_t2i_amd import checkpoints as C
    be, params, shapes = setup
    C.save_infinity_checkpoint(be.es_model.transformer, be.es_model.vae, tmp_path / "shards", tmp_path / "vae.pth",
                               shards=2)
    cfg = InfinityConfig(arch=TINY, pn="0.06M", batches_per_gen=2, micro_batch=0, synthetic_prompt_lens=(5, 40),
                         vae_chunk=8, model_path=str(tmp_path / "shards"), checkpoint_type="torch_shard",
                         vae_path=str(tmp_path / "vae.pth"))
    be2 = InfinityBackend(str(dev), cfg)
    be2.init_and_attach_lora()
    p2, s2 = be2.collect_lora_params()
    assert [tuple(s) for s in s2] == [tuple(s) for s in shapes]
    theta = flatten_params(params).to(dev)
    noiser = EggRollNoiser(shapes, sigma=5e-2, lr_scale=0.1, rank=1, use_antithetic=True)
    tp = noiser.perturb(theta, noiser.epoch_noise(2, seed=4), 2, 0, 2)
    flat = be.step_sampling_info(1)["flat_ids"]
    a = be.generate_population(flat, 1, be.cfg.guidance_scale, tp)
    b = be2.generate_population(flat, 1, be2.cfg.guidance_scale, tp)
    assert torch.equal(a, b)
