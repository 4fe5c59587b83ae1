"""Z-Image-Turbo host (BASELINE configs[3]) on the GPU, tiny architecture: the population forward vs
one member at a time, the bf16 build vs the fp32 restatement of the same architecture with member
factors from theta_k (oracle/zimage_fp32.py), and a full ES epoch at egg rank 4 vs the oracle's
epoch tail.  The architecture restates diffusers' (absent here): parity with diffusers UNPINNED."""
import numpy as np
import pytest
import torch

from hyperscalees_t2i_amd.backend import ZImageBackend, ZImageConfig
from hyperscalees_t2i_amd.es import EggRollNoiser, flatten_params, unflatten_to_params
from hyperscalees_t2i_amd.es_step import ESConfig, ESEngine
from hyperscalees_t2i_amd.rewards import RewardModels
from hyperscalees_t2i_amd.zimage import ZImageArch
from oracle import eggroll_oracle as O

pytestmark = pytest.mark.gpu

TINY = ZImageArch(dim=256, n_layers=2, n_refiner_layers=1, n_heads=2, ffn=512, cap_feat_dim=256, t_mid=256,
                  seq_multiple=16)
PX = 64     # 8 x 8 latent, 16 image tokens


@pytest.fixture(scope="module")
def setup(dev):
    cfg = ZImageConfig(synthetic_weights=True, arch=TINY, vae_widths=(32, 32, 64, 64), width_px=PX, height_px=PX,
                       num_inference_steps=3, batches_per_gen=2, synthetic_prompt_lens=(20, 70))
    be = ZImageBackend(str(dev), cfg)
    be.init_and_attach_lora()
    params, shapes = be.collect_lora_params()
    return be, params, shapes


def test_lora_layout(setup):
    be, params, shapes = setup
    assert len(shapes) == 2 * (4 * 6 + 1)
    assert tuple(shapes[0]) == (2, 256) and tuple(shapes[1]) == (64, 2)


def test_population_forward_matches_single_member(setup, dev):
    be, params, shapes = setup
    theta0 = flatten_params(params).to(dev)
    noiser = EggRollNoiser(shapes, sigma=0.05, lr_scale=0.1, rank=4, use_antithetic=True)
    pop = 3
    tp = noiser.perturb(theta0, noiser.sample_factors(pop, dev, seed=5), pop, 0, pop)
    flat = be.step_sampling_info(1)["flat_ids"]
    imgs = be.generate_population(flat, 1, 0.0, tp).float()
    B = len(flat)
    assert imgs.shape == (pop * B, 3, PX, PX) and torch.isfinite(imgs).all()
    for k in range(pop):
        unflatten_to_params(tp[k], params, shapes)
        one, _ = be.es_model.generate_one_batch([be._dev_prompts[p] for p in flat], seed=1, width_px=PX,
                                                height_px=PX, num_inference_steps=3, output_type="pt")
        a, b = imgs[k * B:(k + 1) * B], one.float()
        rel = ((a - b).norm() / b.norm()).item()
        assert rel < 3e-2, (k, rel)
    unflatten_to_params(theta0, params, shapes)
    assert (imgs[:B] - imgs[B:2 * B]).abs().max().item() > 0      # members really differ


def test_bf16_build_vs_fp32_restatement(setup, dev):
    """Member k's velocity at every step and its decoded images vs the fp32 restatement (same weights,
    same factors, same latents); sigma 5e-2 so the members' LoRA terms are well above bf16 noise.
    Bounds: ~2x the measurement on MI355X (printed; r04u: velocity 0.68 %, image 1.05 %)."""
    from oracle import zimage_fp32 as Z
    be, params, shapes = setup
    theta0 = flatten_params(params).to(dev)
    noiser = EggRollNoiser(shapes, sigma=5e-2, lr_scale=0.1, rank=4, use_antithetic=True)
    pop = 2
    tp = noiser.perturb(theta0, noiser.sample_factors(pop, dev, seed=9), pop, 0, pop)
    info = be.step_sampling_info(2)
    flat = info["flat_ids"]
    uniq = list(dict.fromkeys(flat))
    idx = torch.tensor([uniq.index(f) for f in flat], device=dev)
    embeds = [be._dev_prompts[p] for p in uniq]
    m = be.es_model
    vel = []
    hook = m.transformer.register_forward_hook(lambda _m, _i, o: vel.append(o))
    try:
        imgs = m.generate_population(embeds, idx, tp, 2, 0.0, PX, PX, 3).float()
    finally:
        hook.remove()
    B = len(flat)
    worst = {"vel_rel": 0.0, "img_rel": 0.0}
    for k in range(pop):
        v32, img32 = Z.generate_fp32(m, tp[k], embeds, idx, 2, PX, PX, 3)
        for s in range(3):
            v = vel[s][k * B:(k + 1) * B]
            worst["vel_rel"] = max(worst["vel_rel"], ((v - v32[s]).norm() / v32[s].norm()).item())
        a = imgs[k * B:(k + 1) * B]
        worst["img_rel"] = max(worst["img_rel"], ((a - img32).norm() / img32.norm()).item())
    print("[zimage-fp32]", worst)
    assert worst["vel_rel"] < 0.015 and worst["img_rel"] < 0.02, worst   # measured 0.0068 / 0.0105


def test_engine_step_rank4_matches_oracle(setup, dev):
    be, params, shapes = setup
    rewards = RewardModels.build(dev, tiny=True, synthetic=True)
    theta = flatten_params(params).to(dev)
    pop = 4
    noiser = EggRollNoiser(shapes, sigma=1e-2, lr_scale=1e-1, rank=4, use_antithetic=True)
    eng = ESEngine(be, rewards, noiser, ESConfig(pop_size=pop, egg_rank=4, promptnorm=True, theta_max_norm=40.0), dev)
    new, st = eng.step(theta, seed=3, guidance_scale=0.0)
    eps = noiser.eps_from_factors(noiser.sample_factors(pop, dev, seed=3), pop).cpu().numpy()
    ref, info = O.ref_es_tail(st["_S"].numpy(), eps, theta.cpu().numpy(), promptnorm=True, lr_scale=1e-1,
                              sigma=1e-2, max_step_norm=0.0, theta_max_norm=40.0)
    np.testing.assert_allclose(new.cpu().numpy(), ref, rtol=1e-5, atol=1e-8)
    assert np.array_equal(st["_fitness"]["order"].numpy(), info["order"])
    assert np.isfinite(st["summary/mean_reward"])


@pytest.fixture(scope="module")
def setup_vae_lora(dev):
    """use_vae_decoder_lora=True (es_backend.py:598-608): the decoder's mid-block to_q / to_k / to_v / to_out.0
    carry LoRA too; theta = transformer LoRA then decoder LoRA."""
    cfg = ZImageConfig(synthetic_weights=True, arch=TINY, vae_widths=(32, 32, 64, 64), width_px=PX, height_px=PX,
                       num_inference_steps=3, batches_per_gen=2, synthetic_prompt_lens=(20, 70),
                       use_vae_decoder_lora=True, vae_chunk=4)
    be = ZImageBackend(str(dev), cfg)
    be.init_and_attach_lora()
    params, shapes = be.collect_lora_params()
    return be, params, shapes


def test_vae_decoder_lora_population_vs_single_member_and_fp32(setup_vae_lora, dev):
    """Population decode (each chunk's members' theta rows on the decoder's LoRA'd linears; vae_chunk 4 < the
    8 images per member, so members span several chunks) vs one member at a time with its own LoRA params,
    and vs the fp32 restatement with the decoder LoRA from theta_k; the decoder LoRA really changes the
    images (members differing only in their decoder LoRA decode differently)."""
    from oracle import zimage_fp32 as Z
    be, params, shapes = setup_vae_lora
    theta0 = flatten_params(params).to(dev)
    d_tr = sum(int(np.prod(s)) for s in shapes[:-8])
    noiser = EggRollNoiser(shapes, sigma=5e-2, lr_scale=0.1, rank=4, use_antithetic=True)
    pop = 2
    tp = noiser.perturb(theta0, noiser.epoch_noise(pop, seed=7), pop, 0, pop)
    info = be.step_sampling_info(2)
    flat = info["flat_ids"]
    B = len(flat)
    imgs = be.generate_population(flat, 2, 0.0, tp).float()
    uniq = list(dict.fromkeys(flat))
    idx = torch.tensor([uniq.index(f) for f in flat], device=dev)
    embeds = [be._dev_prompts[p] for p in uniq]
    worst = 0.0
    for k in range(pop):
        unflatten_to_params(tp[k], params, shapes)
        one, _ = be.es_model.generate_one_batch([be._dev_prompts[p] for p in flat], seed=2, width_px=PX, height_px=PX,
                                                num_inference_steps=3, output_type="pt")
        a = imgs[k * B:(k + 1) * B]
        assert ((a - one.float()).norm() / one.float().norm()).item() < 3e-2
        _, img32 = Z.generate_fp32(be.es_model, tp[k], embeds, idx, 2, PX, PX, 3, vae_lora=True)
        worst = max(worst, ((a - img32).norm() / img32.norm()).item())
    unflatten_to_params(theta0, params, shapes)
    print("[zimage-vae-lora] image rel vs fp32", worst)
    assert worst < 0.02, worst
    # only the decoder LoRA differs between two members -> different images
    tp2 = theta0[None].repeat(2, 1)
    tp2[1, d_tr:] += 0.5 * torch.randn(tp2.shape[1] - d_tr, device=dev, generator=torch.Generator(device=dev).manual_seed(1))
    two = be.generate_population(flat, 2, 0.0, tp2).float()
    assert (two[:B] - two[B:]).abs().max().item() > 1e-3


def test_vae_decoder_lora_engine_step_matches_oracle(setup_vae_lora, dev):
    be, params, shapes = setup_vae_lora
    rewards = RewardModels.build(dev, tiny=True, synthetic=True)
    theta = flatten_params(params).to(dev)
    pop = 4
    noiser = EggRollNoiser(shapes, sigma=1e-2, lr_scale=1e-1, rank=4, use_antithetic=True)
    eng = ESEngine(be, rewards, noiser, ESConfig(pop_size=pop, egg_rank=4, promptnorm=True, theta_max_norm=40.0), dev)
    new, st = eng.step(theta, seed=3, guidance_scale=0.0)
    eps = noiser.eps_from_factors(noiser.sample_factors(pop, dev, seed=3), pop).cpu().numpy()
    ref, info = O.ref_es_tail(st["_S"].numpy(), eps, theta.cpu().numpy(), promptnorm=True, lr_scale=1e-1,
                              sigma=1e-2, max_step_norm=0.0, theta_max_norm=40.0)
    np.testing.assert_allclose(new.cpu().numpy(), ref, rtol=1e-5, atol=1e-8)
    assert not np.array_equal(new.cpu().numpy()[-8 * 64:], theta.cpu().numpy()[-8 * 64:])   # decoder LoRA updated


def test_loaded_zimage_generates_identically(dev, tmp_path):
    """A synthetic Z-Image exported as a diffusers directory (checkpoints.save_zimage_diffusers) and loaded
    back through ZImageConfig(model_name=dir) gives a bit-identical population member-eval."""
    from hyperscalees_t2i_amd import checkpoints as C
    arch = ZImageArch(dim=384, n_layers=2, n_refiner_layers=1, n_heads=3, ffn=1024, cap_feat_dim=256, t_mid=1024)
    # 128 px: 8 x 8 = 64 image tokens, a multiple of diffusers' fixed seq_multiple 32 (not in the config)
    kw = dict(width_px=128, height_px=128, num_inference_steps=2, batches_per_gen=2, synthetic_prompt_lens=(20, 70))
    a = ZImageBackend(str(dev), ZImageConfig(synthetic_weights=True, arch=arch, vae_widths=(32, 32, 64, 64), **kw))
    a.init_and_attach_lora()
    C.save_zimage_diffusers(a.es_model.transformer, a.es_model.vae, tmp_path)
    b = ZImageBackend(str(dev), ZImageConfig(model_name=str(tmp_path), **kw))
    b.init_and_attach_lora()
    pa, sa = a.collect_lora_params()
    pb, sb = b.collect_lora_params()
    assert sa == sb
    theta = flatten_params(pa).to(dev)
    noiser = EggRollNoiser(sa, sigma=5e-2, lr_scale=0.1, rank=4, use_antithetic=True)
    tp = noiser.perturb(theta, noiser.epoch_noise(2, seed=1), 2, 0, 2)
    flat = a.step_sampling_info(1)["flat_ids"]
    assert torch.equal(a.generate_population(flat, 1, 0.0, tp), b.generate_population(flat, 1, 0.0, tp))


def test_lora_linear_row_chunks_match_one_launch(dev, monkeypatch):
    """X beyond the GEMMs' 2 GiB operand runs in whole-member row chunks (LoRALinear._forward_chunked):
    with the limit lowered, the chunked population forward equals the one-launch forward, for the plain,
    SiLU-epilogue and gated-residual forms."""
    from hyperscalees_t2i_amd import lora
    m = lora.LoRALinear(256, 320, bias=True, r=2, alpha=8.0).to(dev)
    g = torch.Generator(device=dev).manual_seed(4)
    with torch.no_grad():
        m.weight.copy_(torch.randn(m.weight.shape, generator=g, device=dev) * 0.06)
        m.bias.copy_(torch.randn(320, generator=g, device=dev) * 0.1)
    lora.bind_theta_layout(m)
    n, rpm = 4, 512
    ctx = lora.PopulationContext()
    ctx.theta_pop = torch.randn(n, 2 * 256 + 320 * 2, generator=g, device=dev) * 0.1
    ctx.n_members = n
    lora.set_population(m, ctx)
    x = torch.randn(n * rpm, 256, generator=g, device=dev).bfloat16()
    gate = torch.randn(n * rpm // 256, 320, generator=g, device=dev).bfloat16()
    res0 = torch.randn(n * rpm, 320, generator=g, device=dev).bfloat16()
    want = [m(x), m(x, epi="silu"), m(x, epi="gated", res=res0.clone(), gate=gate, rows_per_group=256)]
    monkeypatch.setattr(lora, "GEMM_OPERAND_LIMIT", 2 * 256 * (2 * rpm))     # one member per chunk
    got = [m(x), m(x, epi="silu"), m(x, epi="gated", res=res0.clone(), gate=gate, rows_per_group=256)]
    lora.set_population(m, None)
    for a, b in zip(got, want):
        assert torch.allclose(a.float(), b.float(), rtol=1e-2, atol=1e-2), (a.float() - b.float()).abs().max()


@pytest.mark.parametrize("rows,heads,tab", [(4 * 96, 2, 96), (777, 30, 777), (64, 3, 16)])
def test_qk_norm_rope_vs_torch(dev, rows, heads, tab):
    """eggroll_qk_norm_rope vs the fp32 torch form (RMS norm * w, then the complex rotation of adjacent
    pairs with the table row = row % tab_rows): within one bf16 rounding of the output."""
    from hyperscalees_t2i_amd import kernels as K
    from oracle.zimage_fp32 import rope
    g = torch.Generator(device=dev).manual_seed(rows)
    x = (torch.randn(rows, heads * 128, generator=g, device=dev) * 3).bfloat16()
    w = (1 + 0.1 * torch.randn(128, generator=g, device=dev)).bfloat16()
    ang = torch.rand(tab, 64, generator=g, device=dev) * 6.3
    cos, sin = torch.cos(ang).contiguous(), torch.sin(ang).contiguous()
    xf = x.float().view(rows, heads, 128)
    y = xf * torch.rsqrt(xf.pow(2).mean(-1, keepdim=True) + 1e-5) * w.float()
    ti = torch.arange(rows, device=dev) % tab
    ref = rope(y[None], cos[ti][None], sin[ti][None])[0].reshape(rows, -1)
    got = K.qk_norm_rope_(x.clone(), w, 1e-5, cos, sin, heads).float()
    err = (got - ref).abs()
    assert (err <= 2 ** -8 * ref.abs() + 1e-6).all(), float(err.max())
