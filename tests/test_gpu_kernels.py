"""HIP kernel parity vs the CPU oracle (and, through injected factors, vs the reference).

Bars: integer/index work bit-exact (Philox words, member->base layout, ranks); fitness kernel
bit-exact vs the oracle's fixed-order restatement; eps/perturb bit-exact for rank 1 (single
product) and <= 2 ulp-ish (rtol 2e-6) otherwise; update within fp32 tolerance (rtol 1e-5);
bf16 LoRA linear within a bf16 tolerance stated per test."""
import math

import numpy as np
import pytest
import torch
import torch.nn.functional as F

from hyperscalees_t2i_amd import _lib, kernels as K
from hyperscalees_t2i_amd.es import EggRollNoiser, paper_prompt_normalized_scores, standardize_fitness
from oracle import eggroll_oracle as O

pytestmark = pytest.mark.gpu

SHAPE_SETS = {
    "lora_small": [(2, 12), (10, 2), (2, 7), (5, 2)],
    "mixed": [(3, 4), (6,), (2, 9), (9, 2), (1, 1)],
}


def _groups(npz):
    keys = {}
    for k in npz.files:
        if "/" in k:
            g, f = k.split("/", 1)
            keys.setdefault(g, {})[f] = npz[k]
    return keys


# ---------------------------------------------------------------------------------- noise
def test_philox_words_bit_exact(dev):
    for seed, j in ((0, 0), (7, 3), (2 ** 40 + 5, 17)):
        got = K.philox_words(seed, j, 4099, dev).cpu().numpy().view(np.uint32)
        assert np.array_equal(got, O.philox_words(seed, j, 4099))


@pytest.mark.parametrize("flen", [1, 7, 4096, 100_003])
def test_noise_factors_match_oracle(dev, flen):
    lay = K.ThetaLayout([(flen,)], 1)
    f = K.noise_factors(11, 5, lay, dev, base_lo=2).cpu().numpy()[:, :flen]
    ref = O.noise_factors(11, 2, 5, flen)
    np.testing.assert_allclose(f, ref, rtol=0, atol=2e-5)


def test_noise_shard_invariance(dev):
    """Base sample j's factors do not depend on which base range generated them."""
    lay = K.ThetaLayout([(2, 2240), (2240, 2)], 1)
    full = K.noise_factors(9, 8, lay, dev)
    part = K.noise_factors(9, 8, lay, dev, base_lo=5)
    assert torch.equal(full[5:], part)
    z = full[:, :lay.factor_len].flatten()
    assert abs(z.mean().item()) < 0.01 and abs(z.std().item() - 1) < 0.01


# ---------------------------------------------------------------------------------- eps / perturb
def test_injected_reference_factors_reproduce_reference_eps(dev, golden):
    g = _groups(golden("g1_eps.npz"))
    for key, d in g.items():
        if key == "meta":
            continue
        sname, rest = key.rsplit("_p", 1)
        pop, rank, anti, _ = rest.split("_")
        pop, rank, anti = int(pop), int(rank[1:]), bool(int(anti[1:]))
        shapes = SHAPE_SETS[sname]
        lay = K.ThetaLayout(shapes, rank)
        fac = torch.from_numpy(lay.pack_factors(d["factors"])).to(dev)
        assert np.array_equal(lay.unpack_factors(fac.cpu().numpy()), d["factors"])
        eps = K.perturb(None, fac, lay, pop, anti, 0, pop, 1.0).cpu().numpy()
        if rank == 1:
            assert np.array_equal(eps, d["eps"]), key
        else:
            np.testing.assert_allclose(eps, d["eps"], rtol=2e-6, atol=1e-7, err_msg=key)
            np.testing.assert_array_equal(eps, O.dev_eps_rows(d["factors"], shapes, pop, rank, anti, 0, pop))
        th = torch.from_numpy(d["theta"]).to(dev)
        tl = K.perturb(th, fac, lay, pop, anti, pop - 1, pop, 0.01).cpu().numpy()[0]
        if rank == 1:
            assert np.array_equal(tl, d["theta_last"]), key
        else:
            np.testing.assert_allclose(tl, d["theta_last"], rtol=2e-6, atol=1e-7, err_msg=key)


def test_perturb_member_ranges_consistent(dev):
    shapes = [(2, 2240), (2240, 2), (2, 256), (13440, 2), (17,)]
    n = EggRollNoiser(shapes, sigma=0.01, lr_scale=0.1, rank=1, use_antithetic=True)
    pop = 9
    fac = n.sample_factors(pop, dev, seed=4)
    theta = torch.randn(n.num_params, device=dev)
    full = n.perturb(theta, fac, pop, 0, pop)
    for lo, hi in ((0, 3), (3, 7), (7, 9)):
        assert torch.equal(n.perturb(theta, fac, pop, lo, hi), full[lo:hi])
    eps = n.eps_from_factors(fac, pop)
    h = pop // 2
    assert torch.equal(eps[:h], -eps[h:2 * h])
    ref = O.dev_eps_rows(n.layout.unpack_factors(fac.cpu().numpy()), shapes, pop, 1, True, 0, pop)
    assert np.array_equal(eps.cpu().numpy(), ref)


# ---------------------------------------------------------------- regenerated (seeded) noise
# eggroll_perturb_seeded / eggroll_update_seeded regenerate every factor value inside the kernel from the
# epoch seed; they must equal the stored path (noise kernel -> perturb / update) bit for bit, on every tile
# kind: fast WIDE / TALL at ranks 1 / 2 / 4 with NU 1 / 2 / 4, aligned 1-D params (VEC4), unaligned 1-D
# params (generic VEC) and rank 3 (generic GEN: a factor element per Philox quad).
SEEDED_SHAPES = [(2, 2240), (2240, 2), (1, 300), (300, 1), (4, 96), (96, 4), (16,), (7,), (3, 5), (5, 3), (2, 7)]


@pytest.mark.parametrize("rank", [1, 2, 3, 4])
@pytest.mark.parametrize("pop,anti", [(8, True), (7, True), (6, False)])
def test_seeded_perturb_bitexact_vs_stored(dev, rank, pop, anti):
    n = EggRollNoiser(SEEDED_SHAPES, sigma=0.01, lr_scale=0.1, rank=rank, use_antithetic=anti)
    theta = torch.randn(n.num_params, device=dev)
    for seed in (3, 2 ** 40 + 11):
        fac = n.sample_factors(pop, dev, seed=seed)
        sf = n.epoch_noise(pop, seed=seed)
        assert torch.equal(sf.materialise(n.layout, dev), fac)
        for lo, hi in ((0, pop), (1, pop - 1)):
            assert torch.equal(n.perturb(theta, sf, pop, lo, hi), n.perturb(theta, fac, pop, lo, hi)), (seed, lo, hi)
        assert torch.equal(n.eps_from_factors(sf, pop, device=dev), n.eps_from_factors(fac, pop))


@pytest.mark.parametrize("rank", [1, 2, 3, 4])
@pytest.mark.parametrize("pop,anti", [(8, True), (7, True), (6, False), (64, True)])
@pytest.mark.parametrize("caps", [(0.0, 0.0), (2e-4, 0.5)])
def test_seeded_update_bitexact_vs_stored(dev, rank, pop, anti, caps):
    n = EggRollNoiser(SEEDED_SHAPES, sigma=0.01, lr_scale=0.1, rank=rank, use_antithetic=anti)
    g = torch.Generator().manual_seed(pop + rank)
    theta = (torch.randn(n.num_params, generator=g) * 0.02).to(dev)
    S = (torch.randn(pop, 4, generator=g) + 20).to(dev)
    fit = K.fitness(S, True)
    fac = n.sample_factors(pop, dev, seed=5)
    a = n.update_from_factors(theta, fac, fit, pop, max_step_norm=caps[0], theta_max_norm=caps[1])
    b = n.update_from_factors(theta, n.epoch_noise(pop, seed=5), fit, pop, max_step_norm=caps[0],
                              theta_max_norm=caps[1])
    assert torch.equal(a, b)


@pytest.mark.parametrize("layout", ["sana_r1_pop64", "zimage_r4_pop128", "infinity_r1_pop32"])
def test_seeded_full_size_layouts_bitexact(dev, layout):
    """The BASELINE node-level configs' theta layouts (one GPU's member share): seeded == stored."""
    from hyperscalees_t2i_amd.model_shapes import infinity_lora_shapes, zimage_turbo_lora_shapes
    from hyperscalees_t2i_amd.sana import SanaArch, sana_lora_shapes
    shapes, rank, pop, nl = {"sana_r1_pop64": (sana_lora_shapes(SanaArch()), 1, 64, 8),
                             "zimage_r4_pop128": (zimage_turbo_lora_shapes(), 4, 128, 16),
                             "infinity_r1_pop32": (infinity_lora_shapes(), 1, 32, 4)}[layout]
    n = EggRollNoiser(shapes, sigma=0.01, lr_scale=0.1, rank=rank, use_antithetic=True)
    theta = torch.randn(n.num_params, device=dev) * 0.01
    fac = n.sample_factors(pop, dev, seed=9)
    sf = n.epoch_noise(pop, seed=9)
    assert torch.equal(n.perturb(theta, sf, pop, pop - nl, pop), n.perturb(theta, fac, pop, pop - nl, pop))
    fit = K.fitness((torch.randn(pop, 4, generator=torch.Generator().manual_seed(2)) + 20).to(dev), True)
    assert torch.equal(n.update_from_factors(theta, sf, fit, pop, theta_max_norm=40.0),
                       n.update_from_factors(theta, fac, fit, pop, theta_max_norm=40.0))


# ---------------------------------------------------------------------------------- fitness
def test_fitness_bit_exact_vs_oracle_and_reference_ranks(dev, golden):
    g = _groups(golden("g2_fitness.npz"))
    for name, d in g.items():
        if name.startswith("z_"):
            continue
        S = torch.from_numpy(d["S"]).to(dev)
        for tag, pn in (("pn", True), ("mean", False)):
            out = {k: v.cpu().numpy() for k, v in K.fitness(S, pn).items()}
            ref = O.dev_fitness(d["S"], pn)
            for k in ("scores", "mu", "fitness", "finite"):
                np.testing.assert_array_equal(out[k], ref[k], err_msg=f"{name}/{tag}/{k}")
            np.testing.assert_array_equal(out["stats"], ref["stats"], err_msg=f"{name}/{tag}/stats")
            assert np.array_equal(out["order"], ref["order"]), f"{name}/{tag} order"
            if f"{tag}_order" in d:  # reference torch.sort ranks
                assert np.array_equal(out["order"], d[f"{tag}_order"]), f"{name}/{tag} ref ranks"


def test_fitness_api_mirrors(dev, golden):
    g = _groups(golden("g2_fitness.npz"))
    d = g["rand_n64_m4"]
    sc, mu, sb = paper_prompt_normalized_scores(torch.from_numpy(d["S"]).to(dev))
    np.testing.assert_allclose(sc.cpu().numpy(), d["pn_scores"], rtol=2e-6, atol=2e-6)
    np.testing.assert_allclose(float(sb), float(d["pn_sigma_bar"]), rtol=1e-6)
    for name in ("z_two", "z_const", "z_rand", "z_one"):
        f = standardize_fitness(torch.from_numpy(g[name]["r"]).to(dev)).cpu().numpy()
        np.testing.assert_allclose(f, g[name]["f"], rtol=2e-5, atol=2e-6, equal_nan=True, err_msg=name)


# ---------------------------------------------------------------------------------- update
@pytest.mark.parametrize("pop,anti,rank", [(8, True, 1), (7, True, 2), (6, False, 1), (64, True, 1), (5, False, 4)])
@pytest.mark.parametrize("caps", [(0.0, 0.0), (0.0, 40.0), (1e-4, 0.0), (0.0, 0.5), (2e-4, 0.5)])
def test_update_matches_reference_formula(dev, pop, anti, rank, caps):
    shapes = [(2, 300), (260, 2), (2, 64), (7,), (96, 2)]
    n = EggRollNoiser(shapes, sigma=0.01, lr_scale=0.1, rank=rank, use_antithetic=anti)
    fac = n.sample_factors(pop, dev, seed=pop)
    g = torch.Generator().manual_seed(pop)
    theta = (torch.randn(n.num_params, generator=g) * 0.02).to(dev)
    S = (torch.randn(pop, 4, generator=g) + 20).to(dev)
    fit = K.fitness(S, True)
    out = n.update_from_factors(theta, fac, fit, pop, max_step_norm=caps[0], theta_max_norm=caps[1])
    eps = n.eps_from_factors(fac, pop).cpu().numpy()
    ref, info = O.ref_es_tail(S.cpu().numpy(), eps, theta.cpu().numpy(), promptnorm=True, lr_scale=0.1, sigma=0.01,
                              max_step_norm=caps[0], theta_max_norm=caps[1])
    np.testing.assert_allclose(out.cpu().numpy(), ref, rtol=1e-5, atol=1e-8)


def test_update_workspace_reuse_and_many_chunks(dev):
    """Repeated calls on ONE update workspace (different caps, a ~2000-chunk layout) each match the
    reference formula: no state leaks from one call's partial sums / scalars into the next."""
    shapes = [(2, 2240), (2240, 2)] * 200 + [(2, 300), (7,)]
    pop = 8
    n = EggRollNoiser(shapes, sigma=0.01, lr_scale=0.1, rank=1, use_antithetic=True)
    fac = n.sample_factors(pop, dev, seed=3)
    g = torch.Generator().manual_seed(3)
    theta = (torch.randn(n.num_params, generator=g) * 0.05).to(dev)
    S = (torch.randn(pop, 4, generator=g) + 20).to(dev)
    fit = K.fitness(S, True)
    eps = n.eps_from_factors(fac, pop).cpu().numpy()
    for caps in [(0.0, 0.0), (1e-4, 0.0), (0.0, 1.0), (0.0, 0.0), (2e-4, 1.0)]:
        out = n.update_from_factors(theta, fac, fit, pop, max_step_norm=caps[0], theta_max_norm=caps[1])
        ref, _ = O.ref_es_tail(S.cpu().numpy(), eps, theta.cpu().numpy(), promptnorm=True, lr_scale=0.1, sigma=0.01,
                               max_step_norm=caps[0], theta_max_norm=caps[1])
        np.testing.assert_allclose(out.cpu().numpy(), ref, rtol=1e-5, atol=1e-8, err_msg=str(caps))


@pytest.mark.parametrize("pop", [128, 7])
def test_update_fitness_vector_at_allocation_end(dev, pop):
    """The fitness vector as the LAST floats of a fresh 2-MiB allocation (where the bench's caching
    allocator had put it when an unclamped fit[2h] scalar load — issued even with no lane in the odd-
    member branch — read past it and faulted): the update reads nothing past fit[pop - 1]."""
    shapes = [(2, 300), (260, 2), (7,)]
    n = EggRollNoiser(shapes, sigma=0.01, lr_scale=0.1, rank=4 if pop % 2 == 0 else 1, use_antithetic=True)
    fac = n.sample_factors(pop, dev, seed=5)
    g = torch.Generator().manual_seed(5)
    theta = (torch.randn(n.num_params, generator=g) * 0.02).to(dev)
    S = (torch.randn(pop, 4, generator=g) + 20).to(dev)
    fit = K.fitness(S, True)
    tail = torch.full((1 << 19,), float("nan"), device=dev)   # exactly 2 MiB: its own segment
    tail[-pop:] = fit["fitness"]
    fit_end = dict(fit, fitness=tail[-pop:])
    for caps in [(0.0, 0.0), (0.0, 40.0)]:
        out = n.update_from_factors(theta, fac, fit_end, pop, max_step_norm=caps[0], theta_max_norm=caps[1])
        torch.cuda.synchronize()
        ref = n.update_from_factors(theta, fac, fit, pop, max_step_norm=caps[0], theta_max_norm=caps[1])
        assert torch.equal(out, ref), caps


def test_update_nonfinite_members(dev):
    shapes = [(2, 40), (40, 2)]
    pop = 8
    n = EggRollNoiser(shapes, sigma=0.01, lr_scale=0.1, rank=1, use_antithetic=True)
    fac = n.sample_factors(pop, dev, seed=1)
    theta = torch.randn(n.num_params, device=dev)
    S = torch.randn(pop, 4, device=dev) + 3
    S[2, 1] = float("nan")
    # promptnorm: one NaN poisons all -> theta unchanged (unifed_es.py:237-240), caps included: a theta
    # whose norm is above theta_max_norm must come back untouched on this early-return path
    fit = K.fitness(S, True)
    assert fit["stats"][1].item() == 0
    assert torch.equal(n.update_from_factors(theta, fac, fit, pop, 0.0, 40.0), theta)
    big = theta * (100.0 / theta.norm())
    assert torch.equal(n.update_from_factors(big, fac, fit, pop, 1e-6, 40.0), big)
    # mean scoring: member 2 dropped, N_f = 7
    fit = K.fitness(S, False)
    out = n.update_from_factors(theta, fac, fit, pop, 0.0, 0.0)
    eps = n.eps_from_factors(fac, pop).cpu().numpy()
    ref, info = O.ref_es_tail(S.cpu().numpy(), eps, theta.cpu().numpy(), promptnorm=False, lr_scale=0.1, sigma=0.01,
                              max_step_norm=0.0, theta_max_norm=0.0)
    assert info["finite"].sum() == 7
    np.testing.assert_allclose(out.cpu().numpy(), ref, rtol=1e-5, atol=1e-8)


# ---------------------------------------------------------------------------------- LoRA linear
def _bf(x):
    return x.to(torch.bfloat16)


def _lora_case(dev, M, N, Kd, r, rpm, bias=True, seed=0):
    g = torch.Generator().manual_seed(seed)
    x = _bf(torch.randn(M, Kd, generator=g)).to(dev)
    W = _bf(torch.randn(N, Kd, generator=g) * 0.05).to(dev)
    b = _bf(torch.randn(N, generator=g)).to(dev) if bias else None
    nm = -(-M // rpm)
    D = r * Kd + N * r + 5
    ld = -(-D // 4) * 4
    tp = (torch.randn(nm, ld, generator=g) * 0.1).to(dev)
    offA, offB = 4, 4 + r * Kd
    return x, W, b, tp, offA, offB


def _lora_ref(x, W, b, tp, offA, offB, r, scale, rpm):
    return O.ref_lora_linear_pop(x.float().cpu().numpy(), W.float().cpu().numpy(),
                                 None if b is None else b.float().cpu().numpy(), tp.cpu().numpy(), offA, offB, r,
                                 scale, rpm)


@pytest.fixture(params=[128, 256, 8, 9, 10, 12],
                ids=["tile128", "tile256", "tile8phase_mfma", "tile8phase_valu", "tile8phase_320", "tile8phase_fused_proj"])
def gemm_tile(request):
    return request.param


@pytest.mark.parametrize("M,N,Kd,r,rpm", [
    (300, 200, 128, 2, 100),      # ragged M, N; members not tile-aligned
    (257, 128, 64, 1, 257),       # single member, one row over a tile
    (1000, 2240, 256, 2, 300),    # Sana cross-attn-like members of 300 rows
    (512, 96, 192, 4, 128),       # r = 4 (VAR-like lora rank)
    (64, 32, 2240, 2, 16),        # proj_out-like N = 32, time-embed rows per member = 16
    (1536, 320, 512, 1, 700),     # r = 1, tiles straddling two members (MFMA epilogue member blocks)
])
def test_lora_linear_pop_vs_fp64(dev, gemm_tile, M, N, Kd, r, rpm):
    x, W, b, tp, offA, offB = _lora_case(dev, M, N, Kd, r, rpm)
    scale = 8.0 / r
    y = K.lora_linear_pop(x, W, b, tp, offA, offB, r, scale, rpm, kernel=gemm_tile)
    torch.cuda.synchronize()
    ref = _lora_ref(x, W, b, tp, offA, offB, r, scale, rpm)
    got = y.float().cpu().numpy()
    # bf16 output rounding (2^-9 relative) + fp32 accumulation over K
    tol = 2 ** -8 * np.abs(ref) + 2e-4 * math.sqrt(Kd) * np.abs(ref).std()
    assert (np.abs(got - ref) <= tol + 1e-3).all(), float(np.abs(got - ref).max())


def test_lora_linear_no_lora_matches_torch_matmul(dev, gemm_tile):
    x, W, b, tp, *_ = _lora_case(dev, 640, 384, 512, 2, 640)
    y = K.lora_linear_pop(x, W, b, None, 0, 0, 0, 0.0, 640, kernel=gemm_tile)
    ref = torch.nn.functional.linear(x.float(), W.float(), b.float())
    assert torch.allclose(y.float(), ref, rtol=1e-2, atol=2e-2)


def test_lora_project_expand_compose(dev):
    M, N, Kd, r, rpm = 600, 320, 256, 2, 200
    x, W, b, tp, offA, offB = _lora_case(dev, M, N, Kd, r, rpm, bias=False)
    base = K.lora_linear_pop(x, W, None, None, 0, 0, 0, 0.0, rpm)
    T = K.lora_project(x, tp, offA, r, rpm)
    fused = K.lora_linear_pop(x, W, None, tp, offA, offB, r, 4.0, rpm)
    two = K.lora_expand(T, tp, offB, r, 4.0, rpm, base.clone())
    assert (fused.float() - two.float()).abs().max().item() <= 0.02 * fused.float().abs().max().item()
    Tref = np.stack([x[i].float().cpu().numpy() @ tp[i // rpm, offA:offA + r * Kd].view(r, Kd).cpu().numpy().T
                     for i in range(M)])
    np.testing.assert_allclose(T.cpu().numpy(), Tref, rtol=1e-4, atol=1e-3)


def test_lora_linear_sana_shape_sampled_rows(dev, gemm_tile):
    """Full Sana attention shape (K = N = 2240) at 2 members x 16384 rows; rows sampled vs fp64."""
    M, N, Kd, r, rpm = 2 * 16384, 2240, 2240, 2, 16384
    x, W, b, tp, offA, offB = _lora_case(dev, M, N, Kd, r, rpm)
    y = K.lora_linear_pop(x, W, b, tp, offA, offB, r, 4.0, rpm, kernel=gemm_tile)
    rows = torch.tensor([0, 1, 127, 128, 5000, 16383, 16384, 16385, 30000, M - 1])
    ref = _lora_ref(x[rows.to(dev)], W, b, tp, offA, offB, r, 4.0, rpm)
    # recompute reference rows with the right member per row
    for i, row in enumerate(rows.tolist()):
        k = row // rpm
        A = tp[k, offA:offA + r * Kd].view(r, Kd).double().cpu().numpy()
        B = tp[k, offB:offB + N * r].view(N, r).double().cpu().numpy()
        ref[i] = O.ref_lora_linear(x[row:row + 1].float().cpu().numpy(), W.float().cpu().numpy(),
                                   b.float().cpu().numpy(), A, B, 4.0)[0]
    got = y[rows.to(dev)].float().cpu().numpy()
    err = np.abs(got - ref)
    assert (err <= 2 ** -8 * np.abs(ref) + 2e-2).all(), float(err.max())


# ---------------------------------------------------------------------------------- dwconv (model op)
@pytest.mark.parametrize("B,H,W,C,ks,pre,glu", [(2, 32, 32, 64, 3, True, True), (3, 7, 5, 64, 3, False, False),
                                                (1, 16, 16, 96, 5, False, False), (2, 9, 11, 64, 5, True, True),
                                                (4, 32, 32, 11200, 3, True, True)])
def test_dwconv_nhwc_vs_torch(dev, B, H, W, C, ks, pre, glu):
    g = torch.Generator().manual_seed(C)
    x = torch.randn(B, H, W, C, generator=g).to(torch.bfloat16).to(dev)
    w = (torch.randn(ks * ks, C, generator=g) / ks).to(torch.bfloat16).to(dev)
    b = torch.randn(C, generator=g).to(torch.bfloat16).to(dev)
    got = K.dwconv_nhwc(x, w, b, ks, pre, glu).float()
    xin = x.float()
    if pre:  # torch semantics: silu on the bf16 tensor returns bf16 (the kernel rounds likewise)
        xin = torch.nn.functional.silu(x).float()
    wc = w.float().t().reshape(C, 1, ks, ks)
    y = torch.nn.functional.conv2d(xin.permute(0, 3, 1, 2), wc, b.float(), padding=ks // 2, groups=C).permute(0, 2, 3, 1)
    if glu:
        a, gt = y.chunk(2, dim=-1)
        y = a * torch.nn.functional.silu(gt)
    err = (got - y).abs()
    assert (err <= 1e-2 * y.abs() + 2e-2).all(), float(err.max())


@pytest.mark.parametrize("B,H,W,C,ks,pre,glu", [(2, 32, 32, 64, 3, True, True), (3, 7, 5, 64, 3, False, False),
                                                (1, 40, 70, 96, 5, False, False), (2, 24, 64, 192, 3, False, True)])
def test_dwconv_block_orders_bitexact(dev, B, H, W, C, ks, pre, glu):
    """The two block orders (1: channel slice fastest, 2: column sweep, incl. an odd slice count and
    ragged bands / tile columns) compute every block identically: bitwise equal outputs, for the
    depthwise conv and the fused depthwise + grouped 1x1."""
    g = torch.Generator().manual_seed(C + H)
    x = torch.randn(B, H, W, C, generator=g).to(torch.bfloat16).to(dev)
    w = (torch.randn(ks * ks, C, generator=g) / ks).to(torch.bfloat16).to(dev)
    b = torch.randn(C, generator=g).to(torch.bfloat16).to(dev)
    y = [K.dwconv_nhwc(x, w, b, ks, pre, glu, kernel=k) for k in (0, 1, 2)]
    assert torch.equal(y[0], y[1]) and torch.equal(y[1], y[2])
    pw = (torch.randn(C // 32, 32, 32, generator=g) / 6).to(torch.bfloat16).to(dev)
    z = [K.dwconv_pw_nhwc(x, w, pw, ks, kernel=k) for k in (0, 1, 2)]
    assert torch.equal(z[0], z[1]) and torch.equal(z[1], z[2])


def test_dwconv_rejects_unsupported_channels(dev):
    from hyperscalees_t2i_amd import _lib
    x = torch.zeros(1, 4, 4, 48, dtype=torch.bfloat16, device=dev)
    w = torch.zeros(9, 48, dtype=torch.bfloat16, device=dev)
    with pytest.raises(_lib.EggrollError, match="multiple of 32"):
        K.dwconv_nhwc(x, w, None, 3, False, False)
    x = torch.zeros(1, 4, 4, 64, dtype=torch.bfloat16, device=dev)
    w = torch.zeros(9, 64, dtype=torch.bfloat16, device=dev)
    with pytest.raises(_lib.EggrollError, match="row stride"):
        K.dwconv_nhwc(x, w, None, 3, False, True, ldo=72)    # cout 32: at most 32 pad channels


@pytest.mark.parametrize("B,H,W,C", [(2, 32, 32, 192), (1, 9, 11, 11200)])
def test_dwconv_padded_output_stride(dev, B, H, W, C):
    """eggroll_dwconv_nhwc_ex: the GLU output written at row stride cout + 32 equals the packed output
    in its first cout channels and is zero in the pad (the buffer starts as NaN, so every pad value
    was written)."""
    g = torch.Generator().manual_seed(C + 1)
    x = torch.randn(B, H, W, C, generator=g).to(torch.bfloat16).to(dev)
    w = (torch.randn(9, C, generator=g) / 3).to(torch.bfloat16).to(dev)
    b = torch.randn(C, generator=g).to(torch.bfloat16).to(dev)
    co = C // 2
    ref = K.dwconv_nhwc(x, w, b, 3, True, True)
    out = torch.full((B, H, W, co + 32), float("nan"), dtype=torch.bfloat16, device=dev)
    got = K.dwconv_nhwc(x, w, b, 3, True, True, out=out, ldo=co + 32)
    assert torch.equal(got[..., :co], ref)
    assert torch.equal(got[..., co:], torch.zeros_like(got[..., co:]))


def test_sana_ffn_point_conv_on_lora_gemm(dev):
    """The Sana FFN (GLUMBConv, hidden 5600 -> K padded to 5632) on the 8-phase GEMM vs the torch
    composition it replaces (F.linear at K = 5600 on hipBLASLt), and its fused gated-residual
    epilogue ("gated32" into the fp32 stream) vs the unfused gated_residual_f32_."""
    from hyperscalees_t2i_amd.sana import GLUMBConv
    B, H, W, D, hid = 2, 16, 16, 2240, 5600
    ff = GLUMBConv(D, hid).to(dev)
    g = torch.Generator(device=dev).manual_seed(3)
    with torch.no_grad():
        for p, s in ((ff.w_inv, D ** -0.5), (ff.w_dw, 1 / 3), (ff.w_point, 0.5 * hid ** -0.5)):
            p.copy_(torch.randn(p.shape, generator=g, device=dev) * s)
        ff.b_inv.copy_(torch.randn(ff.b_inv.shape, generator=g, device=dev) * 0.1)
    x = torch.randn(B, H * W, D, generator=g, device=dev).bfloat16()
    y = ff(x, H, W)
    h = F.silu(F.linear(x, ff.w_inv, ff.b_inv))
    gl = K.dwconv_nhwc(h.view(B, H, W, -1).contiguous(), ff.w_dw, ff.b_dw, 3, pre_silu=False, glu=True)
    ref = F.linear(gl.view(B, H * W, -1).float(), ff.w_point.float())
    err = (y.float() - ref).abs()
    assert (err <= 2 ** -7 * ref.abs() + 1e-2).all(), float(err.max())
    gate = torch.randn(B, D, generator=g, device=dev)
    res = torch.randn(B * H * W, D, generator=g, device=dev)
    want = res.clone()
    K.gated_residual_f32_(want, y.view(-1, D), gate, rows_per_group=H * W)
    got = ff(x, H, W, res=res.clone(), gate=gate)
    assert torch.equal(got, want)


# ---------------------------------------------------------------------------------- fused row ops (model)
@pytest.mark.parametrize("rows,C,strided,add", [(257 * 3, 1280, False, True), (50 * 5, 768, False, True),
                                                (7, 1280, True, True), (33, 64, False, False), (5, 4096, False, True)])
def test_resid_layernorm_vs_torch(dev, rows, C, strided, add):
    """fp32 residual add + LayerNorm -> bf16 (the CLIP towers' pre-norm residual points) vs torch's
    h + y.float(); F.layer_norm(h, w.float(), b.float()).to(bf16): the stream h bit-exact (one fp32 add
    per element), the normalised output within one bf16 rounding (fp32 statistics, summation order
    differs); strided rows = the last layer's [CLS] rows of a [n, T, C] stream."""
    g = torch.Generator().manual_seed(rows + C)
    T = 5 if strided else 1
    base = (torch.randn(rows, T, C, generator=g) * 3 + 0.5).to(dev)
    h = base[:, 0] if strided else base.view(rows, C)
    y = torch.randn(rows, C, generator=g).to(torch.bfloat16).to(dev) if add else None
    w = (1 + 0.3 * torch.randn(C, generator=g)).to(torch.bfloat16).to(dev)
    b = (0.2 * torch.randn(C, generator=g)).to(torch.bfloat16).to(dev)
    h_ref = h + y.float() if add else h.clone()
    ref = torch.nn.functional.layer_norm(h_ref, (C,), w.float(), b.float(), 1e-5)
    out = K.resid_layernorm_(h, y, w, b, 1e-5)
    assert torch.equal(h, h_ref)
    if strided:   # the other rows of the stream are untouched
        assert torch.equal(base[:, 1:], (torch.randn(rows, T, C, generator=torch.Generator().manual_seed(rows + C)) * 3
                                         + 0.5).to(dev)[:, 1:])
    err = (out.float() - ref).abs()
    assert bool((err <= 2.0 ** -8 * ref.abs() + 1e-5).all()), float(err.max())
@pytest.mark.parametrize("C", [32, 128, 256, 512, 1024, 2240, 2560, 4096])
@pytest.mark.parametrize("mode", ["rms_w_b_res", "rms_relu", "layer_adaln"])
def test_rownorm_vs_torch(dev, C, mode):
    g = torch.Generator().manual_seed(C)
    rows, rpg = 96, 24
    x = (torch.randn(rows, C, generator=g) * 2 + 0.5).to(torch.bfloat16).to(dev)
    w = torch.randn(C, generator=g).to(torch.bfloat16).to(dev)
    b = torch.randn(C, generator=g).to(torch.bfloat16).to(dev)
    res = torch.randn(rows, C, generator=g).to(torch.bfloat16).to(dev)
    mods = (torch.randn(rows // rpg, 6, C, generator=g) * 0.3).to(torch.bfloat16).to(dev)
    xf = x.float()
    if mode == "rms_w_b_res":
        got = K.rownorm(x, 1e-5, w=w, b=b, res=res)
        ref = torch.nn.functional.rms_norm(xf, (C,), w.float(), 1e-5) + b.float() + res.float()
    elif mode == "rms_relu":
        got = K.rownorm(x, 1e-5, w=w, act="relu")
        ref = torch.relu(torch.nn.functional.rms_norm(xf, (C,), w.float(), 1e-5))
    else:
        got = K.rownorm(x, 1e-6, layer=True, mscale=mods[:, 1], mshift=mods[:, 0], rows_per_group=rpg)
        sc = mods[:, 1].float().repeat_interleave(rpg, 0)
        sh = mods[:, 0].float().repeat_interleave(rpg, 0)
        ref = torch.nn.functional.layer_norm(xf, (C,), eps=1e-6) * (1 + sc) + sh
    err = (got.float() - ref).abs()
    assert (err <= 1e-2 * ref.abs() + 3e-2).all(), float(err.max())


def test_gated_residual_and_upshortcut(dev):
    g = torch.Generator().manual_seed(3)
    x = torch.randn(4 * 16, 64, generator=g).to(torch.bfloat16).to(dev)
    y = torch.randn(4 * 16, 64, generator=g).to(torch.bfloat16).to(dev)
    mods = torch.randn(4, 6, 64, generator=g).to(torch.bfloat16).to(dev)
    ref = x.float() + mods[:, 2].float().repeat_interleave(16, 0) * y.float()
    K.gated_residual_(x, y, mods[:, 2], rows_per_group=16)
    assert (x.float() - ref).abs().max().item() < 0.05
    for cin, cout in ((64, 64), (64, 32), (32, 16)):
        xs = torch.randn(2, 5, 7, cin, generator=g).to(torch.bfloat16).to(dev)
        ys = torch.randn(2, 10, 14, cout, generator=g).to(torch.bfloat16).to(dev)
        rep = cout * 4 // cin
        sc = torch.nn.functional.pixel_shuffle(xs.permute(0, 3, 1, 2).float().repeat_interleave(rep, dim=1), 2)
        ref = ys.float() + sc.permute(0, 2, 3, 1)
        K.upshortcut_add_(ys, xs)
        assert (ys.float() - ref).abs().max().item() < 0.05


@pytest.mark.parametrize("cin,cout", [(128, 32), (64, 32), (32, 32), (48, 24), (24, 48)])
@pytest.mark.parametrize("with_bias", [False, True])
def test_subpixel_shortcut_bit_exact(dev, cin, cout, with_bias):
    """out[b,2h+i,2w+j,c] = bf16((y4[b,h+i,w+j,(2i+j)*Cout+c] + bias[c]) + x[b,h,w,(4c+2i+j)/rep]),
    rep = 4 Cout / Cin (1, 2, 4 take the vectorised per-low-pixel kernel; 8 the per-output one):
    exact vs a torch restatement of the interleave."""
    g = torch.Generator().manual_seed(cin + cout)
    B, H, W = 2, 5, 7
    x = torch.randn(B, H, W, cin, generator=g).to(torch.bfloat16).to(dev)
    y4 = torch.randn(B, H + 1, W + 1, 4 * cout, generator=g).to(torch.bfloat16).to(dev)
    bias = torch.randn(cout, generator=g).to(torch.bfloat16).to(dev) if with_bias else None
    got = K.subpixel_shortcut(y4, x, bias=bias)
    rep = 4 * cout // cin
    ref = torch.empty(B, 2 * H, 2 * W, cout, dtype=torch.bfloat16, device=dev)
    c = torch.arange(cout, device=dev)
    bf = bias.float() if with_bias else torch.zeros(cout, device=dev)
    for i in range(2):
        for j in range(2):
            k = 2 * i + j
            src = x[:, :, :, (4 * c + k) // rep].float()
            yk = y4[:, i:i + H, j:j + W, k * cout:(k + 1) * cout].float() + bf
            ref[:, i::2, j::2, :] = (yk + src).to(torch.bfloat16)
    assert torch.equal(got, ref)


@pytest.mark.parametrize("cin,cout", [(64, 32), (64, 64), (128, 64)])
def test_subpixel_shortcut_f32(dev, cin, cout):
    """The DC-AE fp32-stream up-block interleave: fp32 shortcut source and output, bf16 shadow = bf16(out);
    the same arithmetic as the bf16 kernel on the fp32 values (exact vs the torch restatement)."""
    g = torch.Generator().manual_seed(cin * cout)
    B, H, W = 2, 5, 7
    x = torch.randn(B, H, W, cin, generator=g).to(dev)
    y4 = torch.randn(B, H + 1, W + 1, 4 * cout, generator=g).to(torch.bfloat16).to(dev)
    bias = torch.randn(cout, generator=g).to(torch.bfloat16).to(dev)
    sh = torch.empty(B, 2 * H, 2 * W, cout, dtype=torch.bfloat16, device=dev)
    got = K.subpixel_shortcut_f32(y4, x, bias=bias, shadow=sh)
    rep = 4 * cout // cin
    ref = torch.empty(B, 2 * H, 2 * W, cout, device=dev)
    c = torch.arange(cout, device=dev)
    for i in range(2):
        for j in range(2):
            k = 2 * i + j
            ref[:, i::2, j::2, :] = (y4[:, i:i + H, j:j + W, k * cout:(k + 1) * cout].float() + bias.float()) \
                + x[:, :, :, (4 * c + k) // rep]
    assert torch.equal(got, ref) and torch.equal(sh, ref.to(torch.bfloat16))


def test_rownorm_fp32_residual_stream(dev):
    """eggroll_rownorm_ex with an fp32 res and fp32 output (the DC-AE fp32 stream, in place) and a bf16
    shadow: out = rms(x) * w + b + res exactly as the bf16-output kernel computes it before rounding."""
    g = torch.Generator(device=dev).manual_seed(11)
    rows, C = 5000, 256
    x = (torch.randn((rows, C), generator=g, device=dev) * 2).to(torch.bfloat16)
    w = (torch.rand(C, generator=g, device=dev) + 0.5).to(torch.bfloat16)
    b = (torch.randn(C, generator=g, device=dev) * 0.1).to(torch.bfloat16)
    r32 = torch.randn((rows, C), generator=g, device=dev)
    sh = torch.empty((rows, C), dtype=torch.bfloat16, device=dev)
    st = r32.clone()
    out = K.rownorm(x, 1e-5, w=w, b=b, res=st, shadow=sh)
    assert out.data_ptr() == st.data_ptr() and out.dtype == torch.float32
    xf = x.float()
    ref = xf * torch.rsqrt(xf.pow(2).mean(-1, keepdim=True) + 1e-5) * w.float() + b.float() + r32
    assert (out - ref).abs().max() <= 1e-5 * ref.abs().max()
    assert torch.equal(sh, out.to(torch.bfloat16))
    # bf16 res -> bf16 output: the unchanged kernel path equals bf16 of the fp32 form with bf16 res
    o16 = K.rownorm(x, 1e-5, w=w, b=b, res=r32.to(torch.bfloat16))
    st2 = r32.to(torch.bfloat16).float()
    o32 = K.rownorm(x, 1e-5, w=w, b=b, res=st2)
    assert torch.equal(o16, o32.to(torch.bfloat16))


@pytest.mark.parametrize("B,H,W", [(2, 37, 21), (1, 64, 64), (1, 136, 18), (3, 9, 100)])  # band walks of 17 / 2 bands
def test_dcae_head_matches_unfused(dev, B, H, W):
    """k_dcae_head (RMSNorm*w+b -> ReLU -> 3x3 conv 128->3 +bias, MFMA) vs the unfused rownorm kernel +
    torch conv2d and vs an fp32 restatement; ragged tiles (37 x 21) exercise the zero halo."""
    from hyperscalees_t2i_amd.dcae import RMSNormC, nchw, nhwc
    g = torch.Generator().manual_seed(H * W)
    x = (torch.randn(B, H, W, 128, generator=g) * 3 + 0.5).to(torch.bfloat16).to(dev)
    with torch.device(dev):
        norm = RMSNormC(128)
    with torch.no_grad():
        norm.weight.copy_((torch.rand(128, generator=g) + 0.5).to(torch.bfloat16))
        norm.bias.copy_((torch.randn(128, generator=g) * 0.2).to(torch.bfloat16))
    w = (torch.randn(3, 128, 3, 3, generator=g) * 0.05).to(torch.bfloat16).to(dev).contiguous(
        memory_format=torch.channels_last)
    cb = (torch.randn(3, generator=g) * 0.1).to(torch.bfloat16).to(dev)
    got = K.dcae_head(x, norm.eps, norm.weight, norm.bias, w, cb).float()
    a = norm(x, act="relu")                                    # bf16 activations, as the kernel stages them
    ref = nhwc(torch.nn.functional.conv2d(nchw(a).float(), w.float(), cb.float(), padding=1))
    err = (got - ref).abs()
    assert (err <= 1e-2 * ref.abs() + 2e-2).all(), float(err.max())
    xf = x.float()
    af = torch.relu(xf * torch.rsqrt(xf.pow(2).mean(-1, keepdim=True) + norm.eps) * norm.weight.float()
                    + norm.bias.float())
    ref32 = nhwc(torch.nn.functional.conv2d(nchw(af), w.float(), cb.float(), padding=1))
    rel = ((got - ref32).norm() / ref32.norm()).item()
    assert rel < 1e-2, rel


@pytest.mark.parametrize("cin,cout,H,W", [(32, 1024, 32, 32), (16, 256, 16, 48)])
def test_conv3x3_small_cin_on_libeggroll(dev, cin, cout, H, W):
    """dcae.Conv3x3 below 64 input channels (the DC-AE conv_in: 32 latent channels -> 1024) runs libeggroll's
    halo conv on channel-padded operands, not MIOpen: vs the fp32 torch conv of the same bf16 operands, and
    the MIOpen path (LIB_SMALL_CIN False) within the same bf16 tolerance."""
    from hyperscalees_t2i_amd import dcae
    g = torch.Generator(device=dev).manual_seed(cin + H)
    with torch.device(dev):
        c = dcae.Conv3x3(cin, cout)
    with torch.no_grad():
        c.weight.copy_((torch.randn(c.weight.shape, generator=g, device=dev) / (9 * cin) ** 0.5).to(torch.bfloat16))
        c.bias.copy_(torch.randn(cout, generator=g, device=dev).to(torch.bfloat16))
    x = torch.randn((2, H, W, cin), generator=g, device=dev).to(torch.bfloat16)
    assert c.lib_small_cin(x)
    got = c(x).float()
    ref = torch.nn.functional.conv2d(x.permute(0, 3, 1, 2).float(), c.weight.float(), c.bias.float(),
                                     padding=1).permute(0, 2, 3, 1)
    assert got.shape == ref.shape
    assert float((got - ref).norm() / ref.norm()) < 4e-3
    assert torch.equal(c(x), c(x))                           # run to run
    lib = c(x)
    try:
        dcae.LIB_SMALL_CIN = False
        miopen = c(x).float()
    finally:
        dcae.LIB_SMALL_CIN = True
    assert float((lib.float() - miopen).norm() / miopen.norm()) < 8e-3


def test_subpixel_upblock_matches_reference(dev):
    """Sub-pixel phase conv + fused interleave/shortcut == nearest-x2 upsample + 3x3 conv + shortcut.
    Widths on both sides of the fused kernel's shape rule (UpBlock.fused_ok): (64, 64), (128, 64) fused; (64, 128)
    (4*Cout / Cin = 8) and (64, 96) (4*Cout % 256 != 0) on the two-launch form instead of an error."""
    from hyperscalees_t2i_amd.dcae import UpBlock
    torch.manual_seed(0)
    for cin, cout, H, W in ((64, 32, 6, 5), (32, 32, 8, 8), (64, 64, 4, 7), (128, 64, 4, 6), (64, 128, 5, 4),
                            (64, 96, 3, 4)):
        with torch.device(dev):
            up = UpBlock(cin, cout)
        with torch.no_grad():
            up.conv.weight.copy_(torch.randn_like(up.conv.weight, dtype=torch.float32) * 0.1)
            up.conv.bias.copy_(torch.randn_like(up.conv.bias, dtype=torch.float32) * 0.1)
        up.refresh_phase_weights()
        x = torch.randn(2, H, W, cin, device=dev).to(torch.bfloat16)
        assert up.fused_ok() == ((cin, cout) in ((64, 64), (128, 64)))
        got = up(x).float()
        ref = up.forward_reference(x).float()
        rel = ((got - ref).norm() / ref.norm()).item()
        assert got.shape == ref.shape and rel < 1e-2, rel


def _linear_attention_ref(q, k, v, relu):
    """fp32 restatement of diffusers SanaLinearAttnProcessor2_0 (q,k,v [B, N, heads, 32])."""
    q, k, v = q.float(), k.float(), v.float()
    if relu:
        q, k = q.clamp_min(0), k.clamp_min(0)
    kv = torch.einsum("bnhj,bnhi->bhij", k, v)
    ks = k.sum(dim=1)                                   # [B, heads, 32]
    num = torch.einsum("bnhj,bhij->bnhi", q, kv)
    den = torch.einsum("bnhj,bhj->bnh", q, ks).unsqueeze(-1)
    return num / (den + 1e-15)


@pytest.mark.parametrize("B,N,heads", [(2, 1024, 3), (3, 300, 2), (1, 17, 1), (2, 4096, 4), (1, 5000, 2)])
def test_linear_attention_separate_qkv(dev, B, N, heads):
    g = torch.Generator().manual_seed(B * N + heads)
    q, k, v = (torch.randn(B, N, heads, 32, generator=g).to(torch.bfloat16).to(dev) for _ in range(3))
    k = k.abs()   # post-ReLU keys, as the Sana attn1 feeds them
    q = q.abs()
    got = K.linear_attention(q.view(B * N, -1), k.view(B * N, -1), v.view(B * N, -1), B, N, heads, 32,
                             relu_qk=False).float().view(B, N, heads, 32)
    ref = _linear_attention_ref(q, k, v, relu=False)
    rel = ((got - ref).norm() / ref.norm()).item()
    assert rel < 8e-3, rel   # bf16 output rounding (2^-8) dominates


def test_linear_attention_interleaved_relu(dev):
    """DC-AE layout: per head h, channels [q | k | v] of 32 each in one [B*N, 3*heads*32] tensor."""
    B, N, heads = 2, 257, 4
    g = torch.Generator().manual_seed(11)
    qkv = torch.randn(B, N, heads, 3, 32, generator=g).to(torch.bfloat16).to(dev)
    flat = qkv.view(B * N, -1)
    got = K.linear_attention(flat, flat[:, 32:], flat[:, 64:], B, N, heads, 96, relu_qk=True)
    ref = _linear_attention_ref(qkv[:, :, :, 0], qkv[:, :, :, 1], qkv[:, :, :, 2], relu=True)
    rel = ((got.float().view(B, N, heads, 32) - ref).norm() / ref.norm()).item()
    assert rel < 8e-3, rel


@pytest.mark.parametrize("B,N,heads,relu", [(8, 16384, 16, True), (32, 1024, 64, False), (4, 16500, 32, True)])
def test_linear_attention_head_pairs_bitexact(dev, B, N, heads, relu):
    """Contiguous heads (hstride 32, even head count: Sana's q / k / v, the DC-AE's planar [Q|K|V]) run as
    head-pair blocks once the per-head grid has >= 8192 blocks (all three shapes); each head's output must
    equal a one-head call on that head's columns (per-head blocks) bit for bit, and the fp32 restatement
    within bf16 rounding.  N >= 8192 takes the 16-tile-per-wave output pass; 16500 ends on partial token
    chunks and a partial output block."""
    g = torch.Generator().manual_seed(B * N + heads)
    inner = heads * 32
    flat = torch.randn(B * N, 3 * inner, generator=g).to(torch.bfloat16).to(dev)
    if not relu:
        flat = flat.abs()   # keep the denominator away from 0 (as Sana's post-ReLU keys)
    q, k, v = flat, flat[:, inner:], flat[:, 2 * inner:]
    got = K.linear_attention(q, k, v, B, N, heads, 32, relu_qk=relu)
    for h in range(heads):
        one = K.linear_attention(q[:, 32 * h:], k[:, 32 * h:], v[:, 32 * h:], B, N, 1, 32, relu_qk=relu)
        assert torch.equal(got[:, 32 * h:32 * h + 32], one), h
    sh = (B, N, heads, 32)
    ref = _linear_attention_ref(q[:, :inner].reshape(sh), k[:, :inner].reshape(sh), v[:, :inner].reshape(sh), relu)
    rel = ((got.float().view(sh) - ref).norm() / ref.norm()).item()
    assert rel < 8e-3, rel


@pytest.mark.parametrize("B,H,W,C,ks", [(2, 9, 13, 96, 5), (1, 64, 64, 384, 5), (2, 20, 40, 64, 3)])
def test_dwconv_pw_vs_torch(dev, B, H, W, C, ks):
    """Fused depthwise conv + grouped 1x1 (groups of 32) vs torch: conv2d(groups=C) in fp32 rounded to
    bf16 (the intermediate the unfused path stores), then the grouped product in fp32."""
    g = torch.Generator().manual_seed(C + ks)
    x = torch.randn(B, H, W, C, generator=g).to(dev, torch.bfloat16)
    wt = (torch.randn(ks * ks, C, generator=g) * 0.2).to(dev, torch.bfloat16)
    pw = (torch.randn(C // 32, 32, 32, generator=g) / math.sqrt(32)).to(dev, torch.bfloat16)
    got = K.dwconv_pw_nhwc(x, wt, pw, ks).float()
    wc = wt.float().t().reshape(C, 1, ks, ks)
    d = torch.nn.functional.conv2d(x.permute(0, 3, 1, 2).float(), wc, padding=ks // 2, groups=C)
    d = d.permute(0, 2, 3, 1).to(torch.bfloat16).float()
    ref = torch.einsum("ngc,goc->ngo", d.reshape(-1, C // 32, 32), pw.float()).reshape(B, H, W, C)
    err = (got - ref).abs()
    # bf16 rounding of the intermediate can flip one ulp between the two fp32 sums; output rounded once
    tol = 2.0 ** -7 * ref.abs() + 2e-3 * ref.abs().max()
    assert bool((err <= tol).all()), f"max err {err.max().item():.3e}"


def test_multiscale_linear_attention_vs_literal(dev):
    """DC-AE SanaMultiscaleLinearAttention (both branches written into column slices of one buffer)
    vs the literal fp32 restatement: qkv proj -> [qkv, grouped-1x1(dw5x5(qkv))] -> ReLU linear
    attention per branch -> concat -> out proj.  The shared RMSNorm+residual tail is applied to both."""
    from hyperscalees_t2i_amd.dcae import MultiscaleLinearAttention
    torch.manual_seed(7)
    c, B, H, W = 128, 2, 9, 13
    m = MultiscaleLinearAttention(c).to(dev)
    with torch.no_grad():
        for p in m.parameters():
            p.copy_((torch.randn_like(p, dtype=torch.float32) * 0.1).to(p.dtype))
    x = torch.randn(B, H, W, c, device=dev).to(torch.bfloat16)
    with torch.no_grad():
        got = m(x).float()
        heads, hd = m.heads, m.hd
        qkv = x.float() @ m.w_qkv.float().t()
        ks = m.scales[0]
        wc = m.ms_dw[0].float().t().reshape(-1, 1, ks, ks)
        d = torch.nn.functional.conv2d(qkv.permute(0, 3, 1, 2), wc, padding=ks // 2,
                                       groups=wc.shape[0]).permute(0, 2, 3, 1)
        p = torch.einsum("ngj,gij->ngi", d.reshape(-1, 3 * heads, hd), m.ms_pw[0].float()).reshape(B, H, W, -1)
        outs = []
        for br in (qkv, p):
            b5 = br.reshape(B, H * W, heads, 3, hd)
            outs.append(_linear_attention_ref(b5[:, :, :, 0], b5[:, :, :, 1], b5[:, :, :, 2], relu=True)
                        .reshape(B, H, W, -1))
        y = torch.cat(outs, dim=-1) @ m.w_out.float().t()
        ref = m.norm_out(y.to(torch.bfloat16), res=x).float()
    rel = ((got - ref).norm() / ref.norm()).item()
    assert rel < 3e-2, rel


def test_multiscale_linear_attention_planar_bitexact(dev):
    """The planar q/k/v relabelling (w_qkv rows, depthwise channels and grouped-1x1 groups permuted
    alike, used at >= PLANAR_MIN_TOKENS tokens) computes every value as the reference layout does:
    bit-identical outputs; the permuted weights refresh when a parameter changes."""
    from hyperscalees_t2i_amd.dcae import MultiscaleLinearAttention
    torch.manual_seed(8)
    c, B, H, W = 128, 2, 16, 24
    m = MultiscaleLinearAttention(c).to(dev)
    with torch.no_grad():
        for p in m.parameters():
            p.copy_((torch.randn_like(p, dtype=torch.float32) * 0.1).to(p.dtype))
    x = torch.randn(B, H, W, c, device=dev).to(torch.bfloat16)
    with torch.no_grad():
        m.PLANAR_MIN_TOKENS = 1 << 30
        ref = m(x)
        m.PLANAR_MIN_TOKENS = 1
        got = m(x)
        assert torch.equal(got, ref)
        m.ms_pw[0].mul_(0.5)
        m.PLANAR_MIN_TOKENS = 1 << 30
        ref2 = m(x)
        m.PLANAR_MIN_TOKENS = 1
        assert torch.equal(m(x), ref2) and not torch.equal(ref2, ref)


def test_bias_act_and_resblock(dev):
    g = torch.Generator().manual_seed(5)
    y = torch.randn(3, 5, 7, 64, generator=g).to(torch.bfloat16).to(dev)
    b = torch.randn(64, generator=g).to(torch.bfloat16).to(dev)
    for act, fn in (("silu", torch.nn.functional.silu), ("relu", torch.relu), (None, lambda t: t)):
        ref = fn(y + b).float()
        got = K.bias_act_(y.clone(), b, act).float()
        assert (got - ref).abs().max().item() <= 0.02 * max(1.0, ref.abs().max().item())


@pytest.mark.parametrize("c", [64, 128, 256])
def test_resblock_matches_reference(dev, c):
    """ResBlock.forward (c = 64: MIOpen + bias/SiLU pass; 128: implicit-GEMM conv on the 512 x 128
    tile; 256: the 256 x 256 tile) vs the literal conv -> SiLU -> conv -> RMSNorm + residual."""
    from hyperscalees_t2i_amd.dcae import ResBlock, conv_gemm_px
    torch.manual_seed(1)
    with torch.device(dev):
        rb = ResBlock(c)
    assert rb.px == conv_gemm_px(c)
    with torch.no_grad():
        for p in rb.parameters():
            p.copy_(torch.randn_like(p, dtype=torch.float32) * (0.05 if p.ndim < 2 else 1.0 / math.sqrt(9 * c)))
    x = torch.randn(2, 9, 6, c, device=dev).to(torch.bfloat16)
    got, ref = rb(x).float(), rb.forward_reference(x).float()
    assert ((got - ref).norm() / ref.norm()).item() < 1e-2


# ---------------------------------------------------------------------------------- implicit-GEMM 3x3 conv
@pytest.mark.parametrize("B,H,W,Cin,Cout,px,bias,act", [
    (2, 16, 16, 64, 64, 1, True, None),
    (2, 16, 32, 128, 128, 2, True, "silu"),
    (1, 7, 10, 128, 128, 2, False, None),     # odd H, tail super-pixel rows (M' % 256 != 0)
    (2, 16, 32, 128, 128, 1, True, "silu"),   # Cout 128 at px 1: the 512 x 128 tile
    (1, 7, 10, 128, 128, 1, False, None),     # 512 x 128 tile with a ragged last tile (70 rows)
    (3, 40, 24, 256, 128, 1, True, None),     # 512 x 128, Cin 256, several tiles + tail (2880 = 5.6 x 512)
    (1, 24, 40, 256, 256, 1, True, "silu"),
    (1, 9, 12, 512, 512, 1, False, None),     # N = 512: two column tiles
    (3, 5, 6, 64, 256, 1, True, None),        # Cin != Cout, tiny image (every pixel is a border pixel)
])
def test_conv3x3_nhwc_vs_torch(dev, B, H, W, Cin, Cout, px, bias, act):
    """eggroll_conv3x3_nhwc vs a torch fp32 conv2d (+bias, +SiLU) on the same bf16 inputs; the kernel
    rounds once to bf16 at the end: |d| <= 2^-8 |y| + 1e-3 max|y|."""
    g = torch.Generator().manual_seed(B * 1000 + H * 10 + px)
    x = torch.randn(B, H, W, Cin, generator=g).to(dev, torch.bfloat16)
    w = (torch.randn(Cout, Cin, 3, 3, generator=g) / math.sqrt(9 * Cin)).to(dev, torch.bfloat16)
    b = (torch.randn(Cout, generator=g) * 0.5).to(dev, torch.bfloat16) if bias else None
    wp = K.pack_conv3x3_weight(w, px)
    y = K.conv3x3_nhwc(x, wp, b.repeat(px) if bias else None, px, act)
    ref = torch.nn.functional.conv2d(x.permute(0, 3, 1, 2).float(), w.float(), b.float() if bias else None, padding=1)
    if act == "silu":
        ref = torch.nn.functional.silu(ref)
    ref = ref.permute(0, 2, 3, 1)
    err = (y.float() - ref).abs()
    tol = 2.0 ** -8 * ref.abs() + 1e-3 * ref.abs().max()
    assert bool((err <= tol).all()), f"max err {err.max().item():.3e} (ref max {ref.abs().max().item():.3e})"


def test_conv3x3_nhwc_rejects_bad_shapes(dev):
    x = torch.zeros(1, 8, 8, 96, device=dev, dtype=torch.bfloat16)   # Cin not a power of two
    w = K.pack_conv3x3_weight(torch.zeros(64, 96, 3, 3, device=dev, dtype=torch.bfloat16), 1)
    with pytest.raises(RuntimeError):
        K.conv3x3_nhwc(x, w, None, 1)


@pytest.mark.parametrize("B,H,W,Cin,px,Cout", [(2, 16, 32, 128, 2, 128), (1, 7, 10, 128, 2, 128), (1, 9, 12, 256, 1, 256),
                                               (2, 5, 6, 64, 1, 256), (2, 16, 32, 128, 1, 128), (1, 7, 10, 128, 1, 128),
                                               (3, 40, 24, 64, 1, 128)])
def test_conv3x3_rmsnorm_nhwc_vs_torch(dev, B, H, W, Cin, px, Cout):
    """conv3x3 -> RMSNorm(* w + b) -> + res in one launch vs torch fp32 on the same bf16 inputs
    (Cout 128 at px 1: the 512 x 128 tile, RMSNorm across its two column waves)."""
    g = torch.Generator().manual_seed(7 + H)
    x = torch.randn(B, H, W, Cin, generator=g).to(dev, torch.bfloat16)
    w = (torch.randn(Cout, Cin, 3, 3, generator=g) / math.sqrt(9 * Cin)).to(dev, torch.bfloat16)
    nw = (1 + 0.2 * torch.randn(Cout, generator=g)).to(dev, torch.bfloat16)
    nb = (0.2 * torch.randn(Cout, generator=g)).to(dev, torch.bfloat16)
    res = torch.randn(B, H, W, Cout, generator=g).to(dev, torch.bfloat16)
    y = K.conv3x3_rmsnorm_nhwc(x, K.pack_conv3x3_weight(w, px), None, px, 1e-5, nw, nb, res).float()
    z = torch.nn.functional.conv2d(x.permute(0, 3, 1, 2).float(), w.float(), None, padding=1).permute(0, 2, 3, 1)
    zn = z * torch.rsqrt(z.pow(2).mean(-1, keepdim=True) + 1e-5) * nw.float() + nb.float()
    ref = zn + res.float()
    err = (y - ref).abs()
    # auto picks the halo kernel where it applies (H % 16 == 0), which rounds the normalised value to
    # bf16 before the residual add (see test_conv3x3_rmsnorm_halo_vs_torch)
    tol = 2.0 ** -7 * (ref.abs() + zn.abs()) + 1e-3 * ref.abs().max()
    assert bool((err <= tol).all()), f"max err {err.max().item():.3e}"


@pytest.mark.parametrize("B,H,W,Cin,Cout,bias,act", [
    (2, 16, 32, 128, 128, True, "silu"),     # 16 x 32 tile (512 x 128), halo = the whole image + pad
    (1, 48, 96, 128, 128, False, None),      # 3 x 3 tiles: interior tiles see real halo pixels
    (2, 32, 64, 64, 128, True, None),        # Cin 64: two 32-channel slices (no middle slice)
    (1, 32, 64, 256, 128, True, "silu"),     # Cin 256 -> 128
    (1, 32, 32, 256, 256, True, None),       # 16 x 16 tile (256 x 256)
    (2, 16, 48, 64, 256, False, "silu"),     # Cin 64 -> 256
    (1, 16, 32, 512, 512, True, None),       # N = 512: two column tiles share each pixel tile
])
@pytest.mark.parametrize("kern", [2, 3])
def test_conv3x3_halo_vs_torch(dev, B, H, W, Cin, Cout, bias, act, kern):
    """Halo-staged conv (512x128 / 256x256 tiles, one 8-wave workgroup per CU; kernel 2: halo rows padded
    to 8 pixels, kernel 3: the unpadded layout) vs torch fp32 on the same bf16 inputs (same bound as the
    tap-staged kernel), vs the tap-staged kernel (1) — both round an fp32 sum once — and kernel 2 == 3
    bitwise (same MFMA sequence, only the LDS layout differs)."""
    g = torch.Generator().manual_seed(B * 100 + H + Cin)
    x = torch.randn(B, H, W, Cin, generator=g).to(dev, torch.bfloat16)
    w = (torch.randn(Cout, Cin, 3, 3, generator=g) / math.sqrt(9 * Cin)).to(dev, torch.bfloat16)
    b = (torch.randn(Cout, generator=g) * 0.5).to(dev, torch.bfloat16) if bias else None
    wp = K.pack_conv3x3_weight(w, 1)
    y = K.conv3x3_nhwc(x, wp, b, 1, act, kernel=kern)
    y1 = K.conv3x3_nhwc(x, wp, b, 1, act, kernel=1)
    ref = torch.nn.functional.conv2d(x.permute(0, 3, 1, 2).float(), w.float(), b.float() if bias else None, padding=1)
    if act == "silu":
        ref = torch.nn.functional.silu(ref)
    ref = ref.permute(0, 2, 3, 1)
    err = (y.float() - ref).abs()
    tol = 2.0 ** -8 * ref.abs() + 1e-3 * ref.abs().max()
    assert bool((err <= tol).all()), f"max err {err.max().item():.3e} (ref max {ref.abs().max().item():.3e})"
    d = (y.float() - y1.float()).abs()
    assert bool((d <= 2.0 ** -7 * ref.abs() + 1e-3 * ref.abs().max()).all())
    assert torch.equal(y, K.conv3x3_nhwc(x, wp, b, 1, act, kernel=5 - kern))


@pytest.mark.parametrize("B,H,W,Cin,Cout,kern", [(2, 16, 32, 128, 128, 2), (1, 32, 64, 64, 128, 2),
                                                  (1, 32, 32, 256, 256, 2), (2, 16, 32, 128, 128, 3),
                                                  (1, 32, 64, 256, 128, 3), (1, 16, 48, 512, 256, 3)])
def test_conv3x3_rmsnorm_halo_vs_torch(dev, B, H, W, Cin, Cout, kern):
    """conv -> RMSNorm -> + res on the halo kernel (2-D tile rows mapped to NHWC pixels)."""
    g = torch.Generator().manual_seed(3 + W)
    x = torch.randn(B, H, W, Cin, generator=g).to(dev, torch.bfloat16)
    w = (torch.randn(Cout, Cin, 3, 3, generator=g) / math.sqrt(9 * Cin)).to(dev, torch.bfloat16)
    nw = (1 + 0.2 * torch.randn(Cout, generator=g)).to(dev, torch.bfloat16)
    nb = (0.2 * torch.randn(Cout, generator=g)).to(dev, torch.bfloat16)
    res = torch.randn(B, H, W, Cout, generator=g).to(dev, torch.bfloat16)
    bias = (0.3 * torch.randn(Cout, generator=g)).to(dev, torch.bfloat16)
    y = K.conv3x3_rmsnorm_nhwc(x, K.pack_conv3x3_weight(w, 1), bias, 1, 1e-5, nw, nb, res, kernel=kern).float()
    z = torch.nn.functional.conv2d(x.permute(0, 3, 1, 2).float(), w.float(), bias.float(), padding=1)
    z = z.permute(0, 2, 3, 1)
    zn = z * torch.rsqrt(z.pow(2).mean(-1, keepdim=True) + 1e-5) * nw.float() + nb.float()
    ref = zn + res.float()
    err = (y - ref).abs()
    # the halo kernel adds the residual to the bf16-rounded normalised value in its store phase (two
    # roundings, as the eager bf16 graph x + norm(conv(h))): the bound covers a rounding of |zn| too
    tol = 2.0 ** -7 * (ref.abs() + zn.abs()) + 1e-3 * ref.abs().max()
    assert bool((err <= tol).all()), f"max err {err.max().item():.3e}"


@pytest.mark.parametrize("B,H,W,Cin,Cout", [
    (2, 64, 32, 128, 128),    # 4 row bands: 4 tiles per workgroup (512 x 128 tile)
    (1, 32, 64, 64, 128),     # 2 bands: 2 tiles per workgroup, Cin 64 (two slices: no middle slice)
    (1, 48, 32, 256, 128),    # 3 bands: 1 tile per workgroup (the chunked epilogue alone)
    (1, 64, 32, 256, 256),    # 256 x 256 tile, 4 tiles per workgroup
    (2, 32, 16, 512, 512),    # N = 512: two column tiles per tile stack
])
def test_conv3x3_halo_multitile_bitexact(dev, B, H, W, Cin, Cout):
    """Kernel 4 (one workgroup streams several vertically stacked tiles: the next tile's halo and first
    weights in flight during the current tile's last slice, C tiles through a dedicated staging region)
    runs the same MFMA sequence per tile as kernel 2: bit-identical outputs, plain / SiLU + bias /
    RMSNorm + residual."""
    g = torch.Generator().manual_seed(H * 7 + Cin)
    x = torch.randn(B, H, W, Cin, generator=g).to(dev, torch.bfloat16)
    w = (torch.randn(Cout, Cin, 3, 3, generator=g) / math.sqrt(9 * Cin)).to(dev, torch.bfloat16)
    b = (torch.randn(Cout, generator=g) * 0.5).to(dev, torch.bfloat16)
    wp = K.pack_conv3x3_weight(w, 1)
    for bias, act in [(None, None), (b, "silu")]:
        y2 = K.conv3x3_nhwc(x, wp, bias, 1, act, kernel=2)
        y4 = K.conv3x3_nhwc(x, wp, bias, 1, act, kernel=4)
        assert torch.equal(y2, y4), (bias is None, act)
    if Cout in (128, 256):
        nw = (1 + 0.2 * torch.randn(Cout, generator=g)).to(dev, torch.bfloat16)
        nb = (0.2 * torch.randn(Cout, generator=g)).to(dev, torch.bfloat16)
        res = torch.randn(B, H, W, Cout, generator=g).to(dev, torch.bfloat16)
        z2 = K.conv3x3_rmsnorm_nhwc(x, wp, b, 1, 1e-5, nw, nb, res, kernel=2)
        z4 = K.conv3x3_rmsnorm_nhwc(x, wp, b, 1, 1e-5, nw, nb, res, kernel=4)
        assert torch.equal(z2, z4)


def test_conv3x3_halo_rejects_ragged(dev):
    x = torch.zeros(1, 8, 8, 64, device=dev, dtype=torch.bfloat16)   # H % 16 != 0
    w = K.pack_conv3x3_weight(torch.zeros(128, 64, 3, 3, device=dev, dtype=torch.bfloat16), 1)
    with pytest.raises(RuntimeError):
        K.conv3x3_nhwc(x, w, None, 1, kernel=2)
    K.conv3x3_nhwc(x, w, None, 1, kernel=0)   # auto falls back to the tap-staged kernel


@pytest.mark.parametrize("B,H,W,Cin,N", [(2, 6, 5, 64, 128), (1, 16, 16, 128, 512), (3, 9, 4, 256, 64)])
def test_conv2x2_pad1_nhwc_vs_torch(dev, B, H, W, Cin, N):
    """ks = 2 implicit-GEMM conv (the up-blocks' sub-pixel phase conv, output (H+1) x (W+1)) vs torch."""
    g = torch.Generator().manual_seed(11 + W)
    x = torch.randn(B, H, W, Cin, generator=g).to(dev, torch.bfloat16)
    w = (torch.randn(N, Cin, 2, 2, generator=g) / math.sqrt(4 * Cin)).to(dev, torch.bfloat16)
    y = K.conv_nhwc(x, K.pack_conv3x3_weight(w, 1), None, 2).float()
    ref = torch.nn.functional.conv2d(x.permute(0, 3, 1, 2).float(), w.float(), None, padding=1).permute(0, 2, 3, 1)
    assert y.shape == ref.shape
    err = (y - ref).abs()
    assert bool((err <= 2.0 ** -8 * ref.abs() + 1e-3 * ref.abs().max()).all()), f"max err {err.max().item():.3e}"


# ---------------------------------------------------------------------------------- full-size properties
@pytest.mark.parametrize("pop", [64, 128])
def test_full_size_sana_layout_properties(dev, pop):
    """BASELINE sizes (Sana-Sprint 1.6B LoRA theta, D = 1,515,456, pop 64 / 128) through size-independent
    properties: antithetic eps pairs are exact negatives; any member range of perturb equals the
    same rows of the full perturb; theta + eps rows == perturb rows; identical score rows for every
    antithetic pair give identical fitness -> every collapsed coefficient is 0 -> theta' == theta
    bit-exact; and the update matches the oracle's reference formula (rtol 1e-5) on random S."""
    from hyperscalees_t2i_amd.sana import sana_lora_shapes
    shapes = sana_lora_shapes()
    n = EggRollNoiser(shapes, sigma=0.01, lr_scale=0.1, rank=1, use_antithetic=True)
    assert n.num_params == 1515456
    fac = n.sample_factors(pop, dev, seed=pop + 1)
    g = torch.Generator().manual_seed(pop)
    theta = (torch.randn(n.num_params, generator=g) * 0.02).to(dev)
    eps = n.eps_from_factors(fac, pop)
    h = pop // 2
    assert torch.equal(eps[:h], -eps[h:])
    lo, hi = pop // 2 - 3, pop // 2 + 5
    part = n.perturb(theta, fac, pop, lo, hi)
    assert torch.equal(part, theta + 0.01 * eps[lo:hi])
    assert torch.equal(part[1:3], n.perturb(theta, fac, pop, lo + 1, lo + 3))
    # paired identical scores -> zero update, bit-exact, at full size
    S_half = torch.randn(h, 4, generator=g) + 20
    fit = K.fitness(torch.cat([S_half, S_half]).to(dev), True)
    assert torch.equal(n.update_from_factors(theta, fac, fit, pop, 0.0, 0.0), theta)
    # random scores: reference formula via the oracle
    S = (torch.randn(pop, 4, generator=g) + 20).to(dev)
    fit = K.fitness(S, True)
    out = n.update_from_factors(theta, fac, fit, pop, 0.0, 40.0)
    ref, _ = O.ref_es_tail(S.cpu().numpy(), eps.cpu().numpy(), theta.cpu().numpy(), promptnorm=True, lr_scale=0.1,
                           sigma=0.01, max_step_norm=0.0, theta_max_norm=40.0)
    np.testing.assert_allclose(out.cpu().numpy(), ref, rtol=1e-5, atol=1e-8)


@pytest.mark.gpu
@pytest.mark.parametrize("r,M,N,Kd,rpm,kernel", [(0, 128 * 257, 5120, 1280, 128 * 257, 8), (0, 777, 200, 128, 777, 8),
                                                 (0, 8192, 2304, 512, 8192, 10), (2, 2 * 8192, 2304, 512, 8192, 8),
                                                 (2, 2 * 8192 + 100, 2240, 2240, 8192, 10)])
def test_lora_linear_pop_gelu_erf_bitexact(dev, r, M, N, Kd, rpm, kernel):
    """Epilogue 8 (exact GELU, the PickScore CLIP-H/14 fc1) == torch's F.gelu of the same kernel's bf16
    output, bit for bit: the CLIP-H shape (128 images x 257 tokens, 1280 -> 5120), ragged M / N, both
    8-phase tiles, with and without the LoRA term."""
    g = torch.Generator(device=dev).manual_seed(M + N + r)
    x = torch.randn((M, Kd), generator=g, device=dev).to(torch.bfloat16)
    W = (torch.randn((N, Kd), generator=g, device=dev) * (2.0 / Kd ** 0.5)).to(torch.bfloat16)
    bias = torch.randn(N, generator=g, device=dev).to(torch.bfloat16)
    tp = torch.randn((-(-M // rpm), Kd * r + N * r + 8), generator=g, device=dev) * 0.05 if r else None
    y = K.lora_gemm(x, W, bias, K.lora_project(x, tp, 0, r, rpm), tp, Kd * r, r, 2.0, rpm, kernel=kernel) if r \
        else K.lora_linear_pop(x, W, bias, None, 0, 0, 0, 0.0, M, kernel=kernel)
    ref = torch.nn.functional.gelu(y)
    out = K.lora_linear_pop_epi(x, W, bias, tp, 0, Kd * r, r, 2.0, rpm, "gelu_erf", kernel=kernel)
    assert float(y.float().abs().max()) > 3.0          # the erf's tails are exercised
    assert torch.equal(out, ref), int((out != ref).sum())


@pytest.mark.parametrize("epi,r,M,N,Kd,rpm", [("silu", 0, 16384, 2304, 512, 16384), ("res", 2, 4 * 4096, 2240, 2240, 4096),
                                             ("gated", 2, 4 * 4096, 2240, 2240, 4096), ("gated", 1, 3 * 1000 + 200, 384, 256, 1000),
                                             ("res", 0, 777, 200, 128, 777), ("gelu", 2, 2 * 8192, 2304, 512, 8192),
                                             ("gelu", 0, 777, 200, 128, 777), ("mul", 2, 4 * 4096, 2240, 2240, 4096),
                                             ("mul", 0, 777, 200, 128, 777)])
def test_lora_linear_pop_epilogue_bitexact(dev, epi, r, M, N, Kd, rpm):
    """eggroll_lora_linear_pop_epi == the same 8-phase GEMM (kernel 8) followed by the separate op it
    fuses (SiLU of the bf16 output / residual add / eggroll_gated_residual), bit for bit; ragged M, N."""
    g = torch.Generator(device=dev).manual_seed(M + N)
    x = torch.randn((M, Kd), generator=g, device=dev).to(torch.bfloat16)
    W = (torch.randn((N, Kd), generator=g, device=dev) / Kd ** 0.5).to(torch.bfloat16)
    bias = torch.randn(N, generator=g, device=dev).to(torch.bfloat16)
    nm = -(-M // rpm)
    tp = torch.randn((nm, Kd * r + N * r + 8), generator=g, device=dev) * 0.05 if r else None
    offA, offB = 0, Kd * r
    y = K.lora_gemm(x, W, bias, K.lora_project(x, tp, offA, r, rpm) if r else None, tp, offB, r, 2.0, rpm, kernel=8) \
        if r else K.lora_linear_pop(x, W, bias, None, 0, 0, 0, 0.0, M, kernel=8)
    res = torch.randn((M, N), generator=g, device=dev).to(torch.bfloat16)
    rpg = 512
    gate = torch.randn((-(-M // rpg), 3 * N), generator=g, device=dev).to(torch.bfloat16)[:, N:2 * N]
    if epi == "silu":
        ref = (y.float() * torch.reciprocal(1.0 + torch.exp(-y.float()))).to(torch.bfloat16)
        out = K.lora_linear_pop_epi(x, W, bias, tp, offA, offB, r, 2.0, rpm, "silu")
        # the device SiLU uses the hardware reciprocal / exp (as the dwconv's): within 1 bf16 ulp of torch,
        # and bitwise equal to the dwconv's own pre-SiLU of the same values
        assert float((out.float() - ref.float()).abs().max()) <= float(ref.float().abs().max()) * 2 ** -7
        w_id = torch.zeros((9, N), device=dev, dtype=torch.bfloat16)
        w_id[4] = 1.0
        pre = K.dwconv_nhwc(y.view(1, 1, M, N), w_id, None, 3, pre_silu=True, glu=False).view(M, N)
        assert torch.equal(out, pre)
        return
    if epi == "gelu":
        # torch's gelu(approximate="tanh") of the bf16 output; the epilogue evaluates it as x * sigmoid(2k)
        # with the hardware exp2 / rcp: at most 1 bf16 ulp apart, 99.8 % equal (measured)
        ref = torch.nn.functional.gelu(y, approximate="tanh")
        out = K.lora_linear_pop_epi(x, W, bias, tp, offA, offB, r, 2.0, rpm, "gelu")
        diff = (out.float() - ref.float()).abs()
        print(f"[gelu-epilogue] bitwise-equal fraction {(diff == 0).float().mean().item():.6f}")
        # (absolute slack for the tiny outputs at x < -2, where torch's 1 + tanh(k) cancels)
        assert (diff <= ref.float().abs() * 2 ** -7 + 1e-5).all(), float(diff.max())
        assert (diff == 0).float().mean().item() > 0.99
        return
    if epi == "mul":
        ref = res * y
        out = K.lora_linear_pop_epi(x, W, bias, tp, offA, offB, r, 2.0, rpm, "mul", res=res.clone())
    elif epi == "res":
        ref = (res.float() + y.float()).to(torch.bfloat16)
        out = K.lora_linear_pop_epi(x, W, bias, tp, offA, offB, r, 2.0, rpm, "res", res=res.clone())
    else:
        ref = K.gated_residual_(res.clone(), y, gate, rows_per_group=rpg)
        out = K.lora_linear_pop_epi(x, W, bias, tp, offA, offB, r, 2.0, rpm, "gated", res=res.clone(), gate=gate,
                                    rows_per_group=rpg)
    assert torch.equal(out, ref)


@pytest.mark.parametrize("M,N,Kd,r,rpm", [(2 * 16384, 2240, 2240, 2, 16384), (3 * 1000 + 200, 2000, 256, 1, 1000),
                                          (777, 200, 128, 0, 777), (4 * 4096, 11200, 640, 0, 4096),
                                          (1536, 320, 64, 2, 700), (2560, 650, 192, 2, 512), (9600, 2240, 2240, 2, 1200)])
def test_gemm_320_tile_bitexact_vs_256(dev, M, N, Kd, r, rpm):
    """Kernel 10 (256 x 320 tile, B halves of 3 + 2 n-fragments) accumulates every output element with
    the same MFMAs in the same k order as kernel 8 (256 x 256): bit-identical outputs, plain and with
    each fused epilogue op; ragged M / N, tiles straddling members, 1 / odd / even K-tile counts."""
    g = torch.Generator(device=dev).manual_seed(M * 7 + N)
    x = torch.randn((M, Kd), generator=g, device=dev).to(torch.bfloat16)
    W = (torch.randn((N, Kd), generator=g, device=dev) / Kd ** 0.5).to(torch.bfloat16)
    bias = torch.randn(N, generator=g, device=dev).to(torch.bfloat16)
    tp = torch.randn((-(-M // rpm), Kd * r + N * r + 8), generator=g, device=dev) * 0.05 if r else None
    offA, offB = 0, Kd * r
    T = K.lora_project(x, tp, offA, r, rpm) if r else None
    y8 = K.lora_gemm(x, W, bias, T, tp, offB, r, 2.0, rpm, kernel=8)
    y10 = K.lora_gemm(x, W, bias, T, tp, offB, r, 2.0, rpm, kernel=10)
    assert torch.equal(y8, y10)
    res = torch.randn((M, N), generator=g, device=dev).to(torch.bfloat16)
    gate = torch.randn((-(-M // 512), N), generator=g, device=dev).to(torch.bfloat16)
    for epi in ("silu", "res", "gated"):
        kw = {} if epi == "silu" else dict(res=res.clone())
        if epi == "gated":
            kw.update(gate=gate, rows_per_group=512)
        o8 = K.lora_linear_pop_epi(x, W, bias, tp, offA, offB, r, 2.0, rpm, epi, kernel=8, **kw)
        kw = {} if epi == "silu" else dict(res=res.clone())
        if epi == "gated":
            kw.update(gate=gate, rows_per_group=512)
        o10 = K.lora_linear_pop_epi(x, W, bias, tp, offA, offB, r, 2.0, rpm, epi, kernel=10, **kw)
        assert torch.equal(o8, o10), epi


@pytest.mark.parametrize("rows,C,rpg", [(3000, 2240, 1000), (777, 128, 100), (64, 96, 64)])
def test_rownorm_fp32_stream_vs_torch(dev, rows, C, rpg):
    """eggroll_rownorm_ex: fp32 residual-stream input and fp32 AdaLN modulation vs the
    torch fp32 formula, output rounded once to bf16; the bf16-input / bf16-modulation form is the
    unchanged eggroll_rownorm (bit-identical to it)."""
    g = torch.Generator(device=dev).manual_seed(rows + C)
    x = torch.randn((rows, C), generator=g, device=dev) * 3 + 0.5
    G = -(-rows // rpg)
    mods = torch.randn((G, 6, C), generator=g, device=dev) * 0.3
    y = K.rownorm(x, 1e-6, layer=True, mscale=mods[:, 1], mshift=mods[:, 0], rows_per_group=rpg)
    gi = torch.arange(rows, device=dev) // rpg
    ref = torch.nn.functional.layer_norm(x, (C,), eps=1e-6) * (1 + mods[gi, 1]) + mods[gi, 0]
    assert y.dtype == torch.bfloat16
    assert (y.float() - ref).abs().max() <= 2 ** -8 * ref.abs().max() + 1e-5
    # bf16 x + bf16 modulation through the new entry point == the old kernel path, bit for bit
    xb, mb = x.to(torch.bfloat16), mods.to(torch.bfloat16)
    a = K.rownorm(xb, 1e-6, layer=True, mscale=mb[:, 1], mshift=mb[:, 0], rows_per_group=rpg)
    out = torch.empty_like(xb)
    from hyperscalees_t2i_amd import _lib
    _lib.call("eggroll_rownorm", xb.data_ptr(), rows, C, 1e-6, 1, None, None, mb[:, 1].data_ptr(), mb[:, 0].data_ptr(),
              6 * C, rpg, 0, None, out.data_ptr(), K._stream(dev))
    assert torch.equal(a, out)


def test_gated_residual_f32(dev):
    """x = fma(gate, y, x) on the fp32 stream (gate fp32 / bf16 / none), bf16 shadow = bf16(x)."""
    g = torch.Generator(device=dev).manual_seed(3)
    rows, C, rpg = 4096, 2240, 1024
    x = torch.randn((rows, C), generator=g, device=dev)
    y = torch.randn((rows, C), generator=g, device=dev).to(torch.bfloat16)
    gate = torch.randn((rows // rpg, 6 * C), generator=g, device=dev)[:, 2 * C:3 * C]
    gi = torch.arange(rows, device=dev) // rpg
    for gt in (gate, gate.to(torch.bfloat16), None):
        x1, sh = x.clone(), torch.empty((rows, C), dtype=torch.bfloat16, device=dev)
        K.gated_residual_f32_(x1, y, gt, rpg, shadow=sh)
        gg = 1.0 if gt is None else gt.double()[gi]
        ref = (x.double() + gg * y.double())
        assert (x1.double() - ref).abs().max() <= 2 ** -23 * ref.abs().max(), gt is None
        assert torch.equal(sh, x1.to(torch.bfloat16))


@pytest.mark.parametrize("kernel", [8, 10])
@pytest.mark.parametrize("epi,r,M,N,Kd,rpm", [("gated32", 2, 4 * 4096, 2240, 2240, 4096), ("res32", 2, 4 * 4096, 2240, 2240, 4096),
                                             ("gated32", 1, 3 * 1000 + 200, 384, 256, 1000), ("res32", 0, 777, 200, 128, 777)])
def test_lora_epilogue_fp32_stream_bitexact(dev, epi, r, M, N, Kd, rpm, kernel):
    """EPI_RES32 / EPI_GATED32 (the fp32 residual stream fused into the store phase of kernel 8 / 10) ==
    the same GEMM followed by eggroll_gated_residual_f32, bit for bit, stream and bf16 shadow; ragged
    shapes."""
    g = torch.Generator(device=dev).manual_seed(M + N + 1)
    x = torch.randn((M, Kd), generator=g, device=dev).to(torch.bfloat16)
    W = (torch.randn((N, Kd), generator=g, device=dev) / Kd ** 0.5).to(torch.bfloat16)
    bias = torch.randn(N, generator=g, device=dev).to(torch.bfloat16)
    tp = torch.randn((-(-M // rpm), Kd * r + N * r + 8), generator=g, device=dev) * 0.05 if r else None
    offA, offB = 0, Kd * r
    y = K.lora_gemm(x, W, bias, K.lora_project(x, tp, offA, r, rpm) if r else None, tp, offB, r, 2.0, rpm, kernel=8) \
        if r else K.lora_linear_pop(x, W, bias, None, 0, 0, 0, 0.0, M, kernel=8)
    res = torch.randn((M, N), generator=g, device=dev)
    rpg = 512
    gate = torch.randn((-(-M // rpg), 3 * N), generator=g, device=dev)[:, N:2 * N]
    ref, ref_sh = res.clone(), torch.empty((M, N), dtype=torch.bfloat16, device=dev)
    K.gated_residual_f32_(ref, y, gate if epi == "gated32" else None, rpg, shadow=ref_sh)
    got, sh = res.clone(), torch.empty((M, N), dtype=torch.bfloat16, device=dev)
    K.lora_linear_pop_epi(x, W, bias, tp, offA, offB, r, 2.0, rpm, epi, res=got, gate=gate if epi == "gated32" else None,
                          rows_per_group=rpg, out=sh, kernel=kernel)
    assert torch.equal(got, ref) and torch.equal(sh, ref_sh)


@pytest.mark.parametrize("epi", ["silu", "gelu", "res", "gated", "mul", "res32", "gated32"])
def test_lora_gemm_epi_with_given_T_bitexact(dev, epi):
    """eggroll_lora_gemm_epi_sel (T precomputed by eggroll_lora_project) == eggroll_lora_linear_pop_epi (which
    runs the same projection + GEMM itself), bit for bit — the pair GemmTimer times apart on the product path."""
    M, N, Kd, r, rpm = 4 * 1024, 640, 512, 2, 1024
    g = torch.Generator(device=dev).manual_seed(7)
    x = torch.randn((M, Kd), generator=g, device=dev).to(torch.bfloat16)
    W = (torch.randn((N, Kd), generator=g, device=dev) / Kd ** 0.5).to(torch.bfloat16)
    bias = torch.randn(N, generator=g, device=dev).to(torch.bfloat16)
    tp = torch.randn((M // rpm, Kd * r + N * r + 8), generator=g, device=dev) * 0.05
    f32 = epi in ("res32", "gated32")
    res = torch.randn((M, N), generator=g, device=dev)
    res = res if f32 else res.to(torch.bfloat16)
    gate = torch.randn((M // 512, N), generator=g, device=dev)
    gate = gate if f32 else gate.to(torch.bfloat16)
    kw = dict(gate=gate if "gated" in epi else None, rows_per_group=512)
    a_res, b_res = (res.clone(), res.clone()) if epi not in ("silu", "gelu") else (None, None)
    a_sh, b_sh = (torch.empty((M, N), dtype=torch.bfloat16, device=dev) for _ in range(2)) if f32 else (None, None)
    a = K.lora_linear_pop_epi(x, W, bias, tp, 0, Kd * r, r, 2.0, rpm, epi, res=a_res, out=a_sh, **kw)
    T = K.lora_project(x, tp, 0, r, rpm)
    b = K.lora_gemm_epi(x, W, bias, T, tp, Kd * r, r, 2.0, rpm, epi, res=b_res, out=b_sh, **kw)
    assert torch.equal(a, b)
    if f32:
        assert torch.equal(a_sh, b_sh)


@pytest.mark.parametrize("B,N,H,L,U,hd", [(4, 64, 2, 37, 2, 112), (3, 100, 3, 300, 3, 112), (6, 17, 1, 320, 2, 112),
                                           (16, 1024, 20, 300, 4, 112),
                                           # the online softmax's key-half boundary (160 of 320 keys; 128 of 256)
                                           (2, 33, 2, 160, 2, 112), (2, 33, 2, 161, 2, 112), (2, 65, 2, 129, 2, 128),
                                           (2, 257, 16, 257, 2, 80),
                                           # Infinity text cross-attention: head dim 128, k / v interleaved in
                                           # one [U*L, 2C] row (mat_kv), -inf masks, rows -> text rows
                                           (8, 36, 4, 77, 4, 128), (6, 145, 2, 256, 3, 128), (5, 1, 3, 20, 2, 128)])
@pytest.mark.parametrize("variant", [0, 1])
def test_cross_attention_vs_sdpa(dev, monkeypatch, B, N, H, L, U, hd, variant):
    """eggroll_cross_attention (MFMA, caption rows through enc_index, additive mask) vs fp32 SDPA on the
    gathered k / v; ragged N, L not a multiple of 16/32, fully-valid and heavily-masked captions.  Both
    kernel forms: 0 = the product's online two-half softmax, 1 = the two-pass form."""
    import torch.nn.functional as F
    monkeypatch.setattr(K, "XATTN_VARIANT", variant)
    g = torch.Generator(device=dev).manual_seed(B * 131 + L)
    q = torch.randn((B * N, H * hd), generator=g, device=dev).to(torch.bfloat16)
    if hd == 128:
        kv = torch.randn((U * L, 2 * H * hd), generator=g, device=dev).to(torch.bfloat16)
        k, v = kv[:, :H * hd], kv[:, H * hd:]
    else:
        k = torch.randn((U * L, H * hd), generator=g, device=dev).to(torch.bfloat16)
        v = torch.randn((U * L, H * hd), generator=g, device=dev).to(torch.bfloat16)
    lens = [L] + [int(x) for x in torch.randint(1, L + 1, (U - 1,), generator=g, device=dev).tolist()]
    bias = torch.zeros((U, L), device=dev, dtype=torch.bfloat16)
    for u, n_valid in enumerate(lens):
        bias[u, n_valid:] = float("-inf") if hd == 128 else -10000.0
    enc_index = torch.arange(B, device=dev) % U if hd != 128 else torch.randint(0, U, (B,), generator=g, device=dev)
    ours = K.cross_attention(q, k, v, B, N, H, hd, L, hd ** -0.5, bias=bias, enc_index=enc_index).float()
    qq = q.view(B, N, H, hd).transpose(1, 2).float()
    kk = k.view(U, L, H, hd)[enc_index].transpose(1, 2).float()
    vv = v.view(U, L, H, hd)[enc_index].transpose(1, 2).float()
    ref = F.scaled_dot_product_attention(qq, kk, vv, attn_mask=bias[enc_index].view(B, 1, 1, L).float(),
                                         scale=hd ** -0.5).transpose(1, 2).reshape(B * N, H * hd)
    rel = float((ours - ref).norm() / ref.norm())
    assert rel < 1e-2, rel     # bf16 P (probabilities rounded before the PV MFMA) + bf16 output
    assert float((ours - ref).abs().max()) < 3e-2 * float(ref.abs().max())


def test_cross_attention_out_of_range_caption_is_nan_not_oob(dev):
    """A device-resident enc_index entry outside [0, U) poisons that image (NaN) without reading past
    k / v; the other images are unaffected.  Host-side checks reject bad shapes and CPU indices."""
    hd, B, N, H, L, U = 112, 3, 16, 2, 40, 2
    g = torch.Generator(device=dev).manual_seed(3)
    q = torch.randn((B * N, H * hd), generator=g, device=dev).to(torch.bfloat16)
    k = torch.randn((U * L, H * hd), generator=g, device=dev).to(torch.bfloat16)
    v = torch.randn((U * L, H * hd), generator=g, device=dev).to(torch.bfloat16)
    good = K.cross_attention(q, k, v, B, N, H, hd, L, 0.1, enc_index=torch.tensor([0, 1, 1], device=dev)).float()
    bad = K.cross_attention(q, k, v, B, N, H, hd, L, 0.1, enc_index=torch.tensor([0, 7, 1], device=dev)).float()
    torch.cuda.synchronize()
    assert torch.isnan(bad[N:2 * N]).all()
    assert torch.equal(bad[:N], good[:N]) and torch.equal(bad[2 * N:], good[2 * N:])
    with pytest.raises(ValueError):
        K.cross_attention(q, k, v, B, N, H, hd, L, 0.1, enc_index=torch.tensor([0, 2, 1]))     # CPU, out of range
    with pytest.raises(ValueError):
        K.cross_attention(q, k, v, B, N, H, hd, L, 0.1)                                        # U < B, no index
    with pytest.raises(ValueError):
        K.cross_attention(q, k, v, B, N, H, hd, L, 0.1, bias=torch.zeros((U, L + 1), device=dev, dtype=torch.bfloat16),
                          enc_index=torch.tensor([0, 1, 1], device=dev))
    # head dim 128 stages at most 256 keys per (text row, head)
    q8 = torch.zeros((2, 128), device=dev, dtype=torch.bfloat16)
    k8 = torch.zeros((257, 128), device=dev, dtype=torch.bfloat16)
    with pytest.raises(_lib.EggrollError, match="L <= 256"):
        K.cross_attention(q8, k8, k8, 2, 1, 1, 128, 257, 0.1, enc_index=torch.tensor([0, 0], device=dev))


@pytest.mark.parametrize("M,Kd,r,n_lin,rpm", [
    (4096, 2240, 2, 3, 1024),   # Sana attn1 q/k/v: K % 128 = 64 tail, members block-aligned
    (1000, 2240, 2, 2, 300),    # attn2 k/v-like: ragged M, members straddling blocks
    (777, 128, 1, 1, 100),      # one linear, rows_per_member not a multiple of 16
    (530, 96, 4, 2, 530),       # K < 128 (tail only), NQ = 8
    (2048, 512, 1, 4, 512),     # 4 linears, NQ = 4
    (300, 160, 3, 1, 17),       # r = 3, tiny members
])
def test_lora_project_multi_vs_fp64_and_single(dev, M, Kd, r, n_lin, rpm):
    """eggroll_lora_project_multi (MFMA, A as bf16 hi + lo) vs fp64 X A^T and vs the per-linear VALU
    projection: both within the hi/lo split's 2^-16 relative error of sum |x| |a| per output."""
    g = torch.Generator().manual_seed(M + Kd)
    x = _bf(torch.randn(M, Kd, generator=g)).to(dev)
    nm = -(-M // rpm)
    offs = [8 + l * (r * Kd + 12) for l in range(n_lin)]
    ld = -(-(offs[-1] + r * Kd + 4) // 4) * 4
    tp = (torch.randn(nm, ld, generator=g) * 0.05).to(dev)
    T = K.lora_project_multi(x, tp, offs, r, rpm)
    torch.cuda.synchronize()
    xs = x.double().cpu()
    tps = tp.double().cpu()
    member = torch.arange(M) // rpm
    for l, off in enumerate(offs):
        A = tps[:, off:off + r * Kd].view(nm, r, Kd)[member]                    # [M, r, K]
        ref = torch.einsum("mk,mqk->mq", xs, A)
        bound = torch.einsum("mk,mqk->mq", xs.abs(), A.abs()) * 2 ** -15 + 1e-6
        got = T[l].double().cpu()
        assert ((got - ref).abs() <= bound).all(), float(((got - ref).abs() / bound).max())
        if r in (1, 2, 3, 4):
            single = K.lora_project(x, tp, off, r, rpm).double().cpu()
            assert ((got - single).abs() <= 2 * bound).all()


def test_lora_project_multi_rejects_bad_args(dev):
    x = torch.zeros((64, 100), dtype=torch.bfloat16, device=dev)
    tp = torch.zeros((1, 1024), device=dev)
    with pytest.raises(K._lib.EggrollError, match="K % 32"):
        K.lora_project_multi(x, tp, [0], 1, 64)                     # K = 100
    x = torch.zeros((64, 128), dtype=torch.bfloat16, device=dev)
    with pytest.raises(K._lib.EggrollError, match="n_lin"):
        K.lora_project_multi(x, tp, [0, 256, 512], 3, 64)           # n_lin * r = 9
    with pytest.raises(K._lib.EggrollError, match="aligned"):
        K.lora_project_multi(x, tp, [2], 1, 64)


@pytest.mark.parametrize("M,Kd,N,r,rpm", [(128, 256, 2240, 2, 16), (37, 2240, 32, 1, 5), (512, 2240, 13440, 2, 64),
                                          (64, 100, 70, 4, 64), (9, 3072, 129, 8, 3), (4096, 2240, 32, 2, 512)])
def test_lora_delta_f32_vs_fp64(dev, M, Kd, N, r, rpm):
    """eggroll_lora_delta_f32 (the fp32 LoRA term of LoRALinear.forward_fp32) vs the PEFT formula in fp64,
    member factors read from a theta_pop column slice (rows member-major, ragged last member); each row equals
    the same row run alone with that member's adapter at member stride 0 (bitwise: a row's reduction order does
    not depend on the member count)."""
    g = torch.Generator(device="cpu").manual_seed(M * 7 + Kd + r)
    n = -(-M // rpm)
    offA, offB = 3, 3 + r * Kd + 5                  # unaligned slices, as theta offsets can be
    ld = offB + N * r + 7
    tp = torch.randn((n, ld), generator=g).to(dev)
    x = torch.randn((M, Kd), generator=g).to(dev)
    base = torch.randn((M, N), generator=g).to(dev)
    scale = 4.0 / r
    y = K.lora_delta_f32(x, tp[:, offA:], ld, tp[:, offB:], ld, r, scale, rpm, base.clone())
    xd, td = x.double(), tp.double()
    want = base.double().clone()
    for k in range(n):
        rows = slice(k * rpm, min(M, (k + 1) * rpm))
        A = td[k, offA:offA + r * Kd].view(r, Kd)
        B = td[k, offB:offB + N * r].view(N, r)
        want[rows] += scale * ((xd[rows] @ A.t()) @ B.t())
    bound = 4e-6 * (xd.abs() @ td[:, offA:offA + r * Kd].abs().view(n, r, Kd).amax(0).t()).amax() \
        * td[:, offB:offB + N * r].abs().amax() * scale * r + 2e-7 * want.abs()
    assert ((y.double() - want).abs() <= bound).all(), float((y.double() - want).abs().max())
    for k in (0, n - 1):                            # the same rows alone, one adapter, stride 0
        rows = slice(k * rpm, min(M, (k + 1) * rpm))
        A = tp[k, offA:offA + r * Kd].contiguous()
        B = tp[k, offB:offB + N * r].contiguous()
        alone = K.lora_delta_f32(x[rows].contiguous(), A, 0, B, 0, r, scale, 1, base[rows].clone())
        assert torch.equal(alone, y[rows])


def test_lora_delta_f32_rejects_bad_args(dev):
    x = torch.zeros((8, 64), device=dev)
    y = torch.zeros((8, 32), device=dev)
    A = torch.zeros(9 * 64, device=dev)
    B = torch.zeros(9 * 32, device=dev)
    with pytest.raises(K._lib.EggrollError, match="r=9"):
        K.lora_delta_f32(x, A, 0, B, 0, 9, 1.0, 8, y)
    with pytest.raises(ValueError, match="too small"):
        K.lora_delta_f32(x, torch.zeros(2 * 64, device=dev), 2 * 64, B, 2 * 32, 2, 1.0, 4, y)  # member 1's A: past the end
    with pytest.raises(K._lib.EggrollError, match="dtype"):
        K.lora_delta_f32(x.bfloat16(), A, 0, B, 0, 1, 1.0, 8, y)
    empty = torch.zeros((0, 32), device=dev)                                   # no rows: a no-op
    assert K.lora_delta_f32(torch.zeros((0, 64), device=dev), A, 0, B, 0, 1, 1.0, 8, empty).shape == (0, 32)


@pytest.mark.parametrize("r", [2, 8, 16])
def test_forward_fp32_any_lora_rank(dev, r):
    """LoRALinear.forward_fp32 at LoRA ranks the bf16 population GEMM accepts (r 16 is above
    eggroll_lora_delta_f32's register budget and takes the bmm form): the population path (rows
    member-major, theta_pop) and the single-member path both equal the PEFT formula in fp64."""
    from hyperscalees_t2i_amd.lora import LoRALinear, PopulationContext
    g = torch.Generator(device="cpu").manual_seed(r)
    Kd, N, n, rpm = 256, 96, 3, 5
    lin = LoRALinear(Kd, N, bias=True, r=r, alpha=2.0 * r).to(dev)
    with torch.no_grad():
        lin.weight.copy_(torch.randn((N, Kd), generator=g).to(dev, torch.bfloat16) * 0.05)
        lin.bias.copy_(torch.randn(N, generator=g).to(dev, torch.bfloat16))
    lin.reset_lora(torch.Generator(device=dev).manual_seed(r), b_std=0.1)
    lin.theta_off_A, lin.theta_off_B = 0, r * Kd
    tp = torch.randn((n, r * Kd + N * r), generator=g).to(dev) * 0.1
    x = torch.randn((n * rpm, Kd), generator=g).to(dev)
    W, b = lin.weight.double(), lin.bias.double()
    lin.ctx = PopulationContext(theta_pop=tp, n_members=n)
    y = lin.forward_fp32(x).double()
    for k in range(n):
        rows = slice(k * rpm, (k + 1) * rpm)
        A, B = tp[k, :r * Kd].double().view(r, Kd), tp[k, r * Kd:].double().view(N, r)
        want = x[rows].double() @ W.t() + b + lin.scale * ((x[rows].double() @ A.t()) @ B.t())
        assert float((y[rows] - want).abs().max()) < 1e-4 * float(want.abs().max()), (r, k)
    lin.ctx = None
    y1 = lin.forward_fp32(x).double()
    A, B = lin.lora_A.weight.double(), lin.lora_B.weight.double()
    want = x.double() @ W.t() + b + lin.scale * ((x.double() @ A.t()) @ B.t())
    assert float((y1 - want).abs().max()) < 1e-4 * float(want.abs().max()), r


def _integration_blocks():
    import re
    from pathlib import Path
    md = (Path(__file__).resolve().parent.parent / "INTEGRATION.md").read_text()
    return re.findall(r"```python\n(.*?)```", md, flags=re.S)


@pytest.mark.parametrize("pop,r,caps", [(8, 1, (0.0, 40.0)), (7, 2, (0.5, 1.0))])
def test_integration_example_runs(dev, pop, r, caps):
    """INTEGRATION.md's ctypes stub + epoch-tail example, executed as documented against the built
    library: theta' equals the package path's (same kernels, bit for bit) and the oracle's epoch tail
    (reference formula on the same factors) within the update's fp32 tolerance."""
    ns = {}
    for blk in _integration_blocks()[:2]:
        exec(blk, ns)
    lib = ns["bind"](str(K._lib.LIB_PATH))
    shapes = [(2, 40), (40, 2), (6,), (2, 12), (33, 2)]
    lay = K.ThetaLayout(shapes, r)
    g = torch.Generator().manual_seed(pop)
    theta = (torch.randn(lay.D, generator=g) * 0.3).to(dev)
    S = torch.randn(pop, 4, generator=g).to(dev)
    max_step, max_theta = caps
    out, theta_pop, factors, fit, order = ns["es_epoch_tail"](lib, shapes, theta, S, epoch=5, pop=pop, r=r,
                                                              sigma=0.01, lr_scale=0.1, theta_max_norm=max_theta,
                                                              max_step_norm=max_step)
    # the package path on the same inputs
    f_pkg = K.noise_factors(5, K.n_base_samples(pop, True), lay, dev)
    fit_pkg = K.fitness(S, True)
    out_pkg = K.update(theta, f_pkg, fit_pkg, lay, pop, True, 0.1 * 0.01, max_step, max_theta)
    pop_pkg = K.perturb(theta, f_pkg, lay, pop, True, 0, pop, 0.01)
    torch.cuda.synchronize()
    assert torch.equal(factors[:, :lay.factor_len], f_pkg[:, :lay.factor_len])
    assert torch.equal(out, out_pkg) and torch.equal(theta_pop, pop_pkg)
    assert torch.equal(order, fit_pkg["order"])
    # the oracle's epoch tail on eps rows built from the same factors
    fac = lay.unpack_factors(factors.cpu().numpy())
    eps = O.dev_eps_rows(fac, shapes, pop, r, True, 0, pop)
    ref, info = O.ref_es_tail(S.cpu().numpy(), eps, theta.cpu().numpy(), promptnorm=True, lr_scale=0.1, sigma=0.01,
                              max_step_norm=max_step, theta_max_norm=max_theta)
    np.testing.assert_allclose(out.cpu().numpy(), ref, rtol=1e-5, atol=1e-7)
    assert np.array_equal(order.cpu().numpy(), info["order"])


@pytest.mark.parametrize("fp32_stages", [0, 4])
def test_dcae_high_res_chunking_is_exact(dev, fp32_stages):
    """DCAEDecoder runs the low-resolution stages on the whole call and the two high-resolution stages in
    chunks of hi_res_chunk images: the result equals decoding each chunk on its own (to GEMM-library
    reduction order: hipBLASLt may pick another kernel for another row count)."""
    from hyperscalees_t2i_amd.dcae import DCAEDecoder
    vae = DCAEDecoder(32, widths=(16, 32, 32, 64, 64, 64), layers=(1, 1, 1, 1, 1, 1)).to(dev)
    vae.init_weights(3)
    vae.fp32_stages = fp32_stages
    z = torch.randn(6, 32, 2, 2, generator=torch.Generator().manual_seed(5)).to(dev)
    with torch.no_grad():
        vae.hi_res_chunk = 2
        got = vae(z)
        vae.hi_res_chunk = 8
        want = torch.cat([vae(z[s:s + 2]) for s in range(0, 6, 2)])
    assert got.shape == want.shape
    assert (got.float() - want.float()).abs().max().item() < 3e-2


@pytest.mark.parametrize("B,Nq,Lk,H,strided", [(2, 676, 676, 3, False), (3, 1, 1, 2, False), (2, 100, 2521, 2, True),
                                               (1, 257, 130, 1, True), (4, 64, 64, 2, False)])
def test_flash_attention_vs_sdpa(dev, B, Nq, Lk, H, strided):
    """eggroll_flash_attention (head dim 128, online softmax over 64-key blocks, P in bf16 for the PV MFMA) vs
    fp32 SDPA on the same bf16 inputs; k / v optionally a slice of a longer [B, ltot, H*128] cache (batch
    stride != rows * row stride), ragged query / key counts."""
    g = torch.Generator(device=dev).manual_seed(Nq * 7 + Lk)
    q = (torch.randn(B, Nq, H, 128, generator=g, device=dev) * 0.3).bfloat16()
    if strided:
        cache = (torch.randn(2, B, Lk + 37, H * 128, generator=g, device=dev) * 0.3).bfloat16()
        k = cache[0, :, :Lk].view(B, Lk, H, 128)
        v = cache[1, :, :Lk].view(B, Lk, H, 128)
    else:
        k = (torch.randn(B, Lk, H, 128, generator=g, device=dev) * 0.3).bfloat16()
        v = torch.randn(B, Lk, H, 128, generator=g, device=dev).bfloat16()
    scale = 128 ** -0.5 * 3
    got = K.flash_attention(q, k, v, scale).float()
    ref = torch.nn.functional.scaled_dot_product_attention(q.float().transpose(1, 2), k.float().transpose(1, 2),
                                                           v.float().transpose(1, 2), scale=scale).transpose(1, 2)
    err = ((got - ref).norm() / ref.norm()).item()
    assert err < 1e-2, err
    assert (got - ref).abs().max().item() < 0.05


@pytest.mark.parametrize("B,H,W,C,G,silu", [(2, 48, 40, 128, 32, True), (3, 17, 9, 160, 32, False), (1, 64, 64, 640, 32, True),
                                            (2, 5, 7, 64, 8, True)])
def test_group_norm_nhwc_vs_torch(dev, B, H, W, C, G, silu):
    """eggroll_group_norm_nhwc vs fp32 torch.group_norm (+ silu) on the same bf16 input: within one bf16
    rounding of the output (the stats are fp32 partial sums combined in fp64, torch's are Welford)."""
    from hyperscalees_t2i_amd import kernels as Kk
    g = torch.Generator(device=dev).manual_seed(C + H)
    x = (torch.randn(B, H, W, C, generator=g, device=dev) * 3 + 1.5).bfloat16()
    w = (1 + 0.2 * torch.randn(C, generator=g, device=dev)).bfloat16()
    b = (0.3 * torch.randn(C, generator=g, device=dev)).bfloat16()
    ref = torch.nn.functional.group_norm(x.float().permute(0, 3, 1, 2), G, w.float(), b.float(), 1e-6)
    if silu:
        ref = torch.nn.functional.silu(ref)
    ref = ref.permute(0, 2, 3, 1)
    got = Kk.group_norm_nhwc(x, G, w, b, 1e-6, silu=silu).float()
    err = (got - ref).abs()
    assert (err <= ref.abs() * 2 ** -7 + 2e-3).all(), float(err.max())


@pytest.mark.gpu
@pytest.mark.parametrize("M_img,H,W,C,H2,ldo", [(2, 8, 8, 64, 512, 0), (2, 4, 8, 128, 384, 224)])
def test_glumbconv_silu_placement_bitexact(dev, M_img, H, W, C, H2, ldo):
    """GLUMBConv's SiLU in the inverted conv's GEMM epilogue (lora.SILU_IN_GEMM) and in the depthwise
    conv's staging (the default since round 5) compute silu of the same bf16-rounded GEMM output with
    the same device silu: the depthwise conv outputs are bitwise equal."""
    g = torch.Generator(device=dev).manual_seed(5)
    M = M_img * H * W
    x = (torch.randn(M, C, device=dev, generator=g) * 0.5).bfloat16()
    wi = (torch.randn(H2, C, device=dev, generator=g) * C ** -0.5).bfloat16()
    bi = (torch.randn(H2, device=dev, generator=g) * 0.1).bfloat16()
    wd = (torch.randn(9, H2, device=dev, generator=g) * 0.2).bfloat16()
    bd = (torch.randn(H2, device=dev, generator=g) * 0.1).bfloat16()
    h_epi = K.lora_linear_pop_epi(x, wi, bi, None, 0, 0, 0, 0.0, M, "silu")
    a = K.dwconv_nhwc(h_epi.view(M_img, H, W, H2), wd, bd, 3, pre_silu=False, glu=True, ldo=ldo)
    h = K.lora_linear_pop(x, wi, bi, None, 0, 0, 0, 0.0, M)
    b = K.dwconv_nhwc(h.view(M_img, H, W, H2), wd, bd, 3, pre_silu=True, glu=True, ldo=ldo)
    assert torch.equal(a, b)


@pytest.mark.gpu
@pytest.mark.parametrize("cin,cout,B,H,W", [(256, 128, 2, 12, 20), (128, 128, 1, 9, 7), (64, 64, 2, 5, 6),
                                            (128, 64, 1, 8, 8), (256, 64, 2, 7, 11), (512, 256, 1, 16, 16)])
@pytest.mark.parametrize("f32", [False, True])
def test_conv2x2_subpixel_fused_bitexact(dev, cin, cout, B, H, W, f32):
    """The up-block phase conv with the interleave + bias + shortcut in its epilogue
    (eggroll_conv2x2_subpixel_nhwc, REP = 4 Cout / Cin in {1, 2, 4}) == conv_nhwc(ks 2) followed by
    subpixel_shortcut / subpixel_shortcut_f32, bitwise (bf16 stream, and the fp32 stream + shadow);
    ragged positions (H, W not tile multiples) and the dropped border positions of the phase grid."""
    from hyperscalees_t2i_amd.dcae import subpixel_phase_weights
    g = torch.Generator(device=dev).manual_seed(cin + cout + H)
    w3 = torch.randn(cout, cin, 3, 3, device=dev, generator=g) * (9 * cin) ** -0.5
    w4 = subpixel_phase_weights(w3).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    wp = K.pack_conv3x3_weight(w4, 1)
    bias = (torch.randn(cout, device=dev, generator=g) * 0.1).bfloat16()
    x = torch.randn(B, H, W, cin, device=dev, generator=g).bfloat16()
    y4 = K.conv_nhwc(x, wp, None, 2)
    if f32:
        x32 = x.float() + torch.randn(B, H, W, cin, device=dev, generator=g) * 1e-3
        s_ref = torch.empty(B, 2 * H, 2 * W, cout, device=dev, dtype=torch.bfloat16)
        ref = K.subpixel_shortcut_f32(y4, x32, bias=bias, shadow=s_ref)
        s_got = torch.empty_like(s_ref)
        got = K.conv2x2_subpixel(x, wp, x32, bias=bias, shadow=s_got)
        assert torch.equal(got, ref) and torch.equal(s_got, s_ref)
    else:
        ref = K.subpixel_shortcut(y4, x, bias=bias)
        got = K.conv2x2_subpixel(x, wp, x, bias=bias)
        assert torch.equal(got, ref)
