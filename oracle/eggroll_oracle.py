"""CPU oracle: numpy restatement of the reference EGGROLL ES hot path.

TEST INFRASTRUCTURE ONLY.  Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline
leg may import this module, and only as the checker / the timed CPU baseline.  The product
path (hyperscalees_t2i_amd) never imports it and fails loudly without libeggroll.so.

Reference: amit154154/HyperscaleES_T2I (pure Python).  Every function cites the lines it
restates.  Parity is PINNED: tests/test_oracle_golden.py checks this module against golden
vectors produced by the reference's own `utills.py` (imported in the build container by
tests/golden/make_golden.py; fixtures committed under tests/golden/).  The PEFT LoRA-linear
formula (third-party `peft`, unpinned version, not vendored) is restated from its published
algorithm and is "parity unpinned" beyond that formula.

Two families of functions live here:
  * `ref_*`  follow the reference's op order (torch semantics) and are compared with the
             golden vectors within fp32 tolerance;
  * `dev_*`  restate the same algorithm in the FIXED sequential fp32 op order that the HIP
             kernels use, so kernel-vs-oracle comparisons can be bit-exact.
"""
from __future__ import annotations

import math
from typing import Dict, List, Sequence, Tuple

import numpy as np

F32 = np.float32
NOISE_TAG = np.uint32(0xE6606011)
CHUNK = 1024

# ---------------------------------------------------------------------------------------
# indexing (utills.py:364-379, es_backend.py:234-263) — bit-exact integer work
# ---------------------------------------------------------------------------------------


def sample_indices_unique(seed: int, total: int, k: int) -> List[int]:
    """utills.py:364-373."""
    if total <= 0:
        raise ValueError("total must be >= 1")
    if k <= 0:
        raise ValueError("k must be >= 1")
    rng = np.random.RandomState(int(seed))
    if k >= total:
        return list(range(total))
    return rng.choice(np.arange(total, dtype=np.int64), size=k, replace=False).tolist()


def repeat_batches(ids_unique: Sequence[int], repeats: int) -> List[int]:
    """utills.py:376-379 (prompt-major inner order)."""
    if repeats <= 0:
        raise ValueError("repeats must be >= 1")
    return [i for _ in range(repeats) for i in ids_unique]


def member_to_base(k: int, pop: int, antithetic: bool) -> Tuple[int, float]:
    """Antithetic layout of EggRollNoiser.sample_eps (utills.py:88-105)."""
    if not antithetic:
        return k, 1.0
    h = pop // 2
    if k < h:
        return k, 1.0
    if k < 2 * h:
        return k - h, -1.0
    return h, 1.0


def n_base_samples(pop: int, antithetic: bool) -> int:
    """utills.py:88-89: base_pop = half (+1 if odd)."""
    return (pop // 2 + pop % 2) if antithetic else pop


# ---------------------------------------------------------------------------------------
# theta layout (utills.py:141-162)
# ---------------------------------------------------------------------------------------


def _pad4(x: int) -> int:
    return -(-x // 4) * 4


def layout(shapes: Sequence[Sequence[int]], rank: int) -> Dict[str, object]:
    """theta = concat(p.view(-1)) in parameter order; factors per base sample = for each
    matrix a [m][r] then b [n][r]; 1-D params: numel dense values.  The device buffer pads every
    segment to a multiple of 4 floats (include/eggroll.h); the functions below that take factor
    arrays use the reference's contiguous order (ThetaLayout.unpack_factors converts)."""
    recs = []
    toff = foff = coff = 0
    for s in shapes:
        s = tuple(int(x) for x in s)
        if len(s) == 2:
            m, n = s
            numel, fl = m * n, _pad4(rank * m) + _pad4(rank * n)
        else:
            m, n = int(np.prod(s)), 0
            numel, fl = m, _pad4(m)
        recs.append((m, n, toff, foff, coff, 0))
        toff += numel
        foff += fl
        coff += -(-numel // CHUNK)
    return {"mats": np.array(recs, dtype=np.int64).reshape(-1, 6), "D": toff, "factor_len": foff,
            "total_chunks": coff}


# ---------------------------------------------------------------------------------------
# (1) noise: Philox4x32-10 + Box-Muller, counter = (g/4, j, NOISE_TAG), key = seed
# ---------------------------------------------------------------------------------------

_M0, _M1 = np.uint64(0xD2511F53), np.uint64(0xCD9E8D57)
_W0, _W1 = np.uint32(0x9E3779B9), np.uint32(0xBB67AE85)
_MASK = np.uint64(0xFFFFFFFF)


def philox4x32_10(c0, c1, c2, c3, k0: int, k1: int):
    """Salmon et al. SC'11, Random123 constants; vectorised over counters (uint32 arrays)."""
    c0, c1, c2, c3 = (np.asarray(x, dtype=np.uint32).copy() for x in (c0, c1, c2, c3))
    k0 = np.uint32(k0)
    k1 = np.uint32(k1)
    with np.errstate(over="ignore"):
        for _ in range(10):
            p0 = _M0 * c0.astype(np.uint64)
            p1 = _M1 * c2.astype(np.uint64)
            hi0, lo0 = (p0 >> np.uint64(32)).astype(np.uint32), (p0 & _MASK).astype(np.uint32)
            hi1, lo1 = (p1 >> np.uint64(32)).astype(np.uint32), (p1 & _MASK).astype(np.uint32)
            c0, c1, c2, c3 = hi1 ^ c1 ^ k0, lo1, hi0 ^ c3 ^ k1, lo0
            k0 = np.uint32(k0 + _W0)
            k1 = np.uint32(k1 + _W1)
    return c0, c1, c2, c3


def philox_words(seed: int, j: int, n_quads: int) -> np.ndarray:
    q = np.arange(n_quads, dtype=np.uint64)
    w = philox4x32_10((q & _MASK).astype(np.uint32), (q >> np.uint64(32)).astype(np.uint32),
                      np.full(n_quads, j, np.uint32), np.full(n_quads, NOISE_TAG, np.uint32),
                      seed & 0xFFFFFFFF, (seed >> 32) & 0xFFFFFFFF)
    return np.stack(w, axis=1).reshape(-1)


def _box_muller(w0: np.ndarray, w1: np.ndarray):
    u1 = ((w0 >> np.uint32(9)).astype(F32) + F32(0.5)) * F32(2.0 ** -23)
    u2 = (w1 >> np.uint32(9)).astype(F32) * F32(2.0 ** -23)
    rr = np.sqrt(F32(-2.0) * np.log(u1.astype(np.float64)).astype(F32)).astype(F32)
    ang = np.float64(np.pi) * (F32(2.0) * u2).astype(np.float64)
    return (rr * np.cos(ang).astype(F32)).astype(F32), (rr * np.sin(ang).astype(F32)).astype(F32)


def noise_factors(seed: int, base_lo: int, base_hi: int, factor_len: int) -> np.ndarray:
    """Device noise restated: out[j - base_lo, g] ~ N(0,1).  Matches the kernel's Philox words
    bit-exactly and its normals to ~1e-6 (libm transcendental ulps)."""
    nq = -(-factor_len // 4)
    out = np.empty((base_hi - base_lo, nq * 4), F32)
    for j in range(base_lo, base_hi):
        w = philox_words(seed, j, nq).reshape(nq, 4)
        z0, z1 = _box_muller(w[:, 0], w[:, 1])
        z2, z3 = _box_muller(w[:, 2], w[:, 3])
        out[j - base_lo] = np.stack([z0, z1, z2, z3], axis=1).reshape(-1)
    return out[:, :factor_len]


# ---------------------------------------------------------------------------------------
# eps from factors (utills.py:43-106): E = (A @ B^T) / sqrt(r); antithetic cat layout
# ---------------------------------------------------------------------------------------


def split_factors(factors: np.ndarray, shapes, rank: int):
    """factor vector(s) [p, factor_len] -> list of (A [p,m,r], B [p,n,r]) or dense [p,numel]."""
    out = []
    off = 0
    p = factors.shape[0]
    for s in shapes:
        if len(s) == 2:
            m, n = int(s[0]), int(s[1])
            a = factors[:, off:off + m * rank].reshape(p, m, rank)
            off += m * rank
            b = factors[:, off:off + n * rank].reshape(p, n, rank)
            off += n * rank
            out.append((a, b))
        else:
            numel = int(np.prod(s))
            out.append(factors[:, off:off + numel])
            off += numel
    return out


def ref_eps_from_blocks(blocks, shapes, pop: int, rank: int, antithetic: bool) -> np.ndarray:
    """utills.py:50-68 + 70-106 in the reference's op order (fp32)."""
    chunks = []
    for blk, s in zip(blocks, shapes):
        if len(s) == 2:
            a, b = blk
            e = np.matmul(a.astype(F32), np.swapaxes(b.astype(F32), 1, 2)).astype(F32) / F32(math.sqrt(rank))
            chunks.append(e.reshape(e.shape[0], -1).astype(F32))
        else:
            chunks.append(blk.astype(F32))
    base = np.concatenate(chunks, axis=1)
    if not antithetic:
        return base[:pop]
    half = pop // 2
    eps = np.concatenate([base[:half], -base[:half]], axis=0)
    if pop % 2 == 1:
        eps = np.concatenate([eps, base[half:half + 1]], axis=0)
    return eps


def dev_eps_rows(factors: np.ndarray, shapes, pop: int, rank: int, antithetic: bool,
                 member_lo: int, member_hi: int) -> np.ndarray:
    """Kernel op order: E[i,c] = (sum_q a[i,q]*b[c,q] sequential, no fma) / float(sqrt(r))."""
    sqrt_r = F32(math.sqrt(rank))
    blocks = split_factors(factors, shapes, rank)
    rows = []
    for k in range(member_lo, member_hi):
        j, sgn = member_to_base(k, pop, antithetic)
        parts = []
        for blk, s in zip(blocks, shapes):
            if len(s) == 2:
                a, b = blk[0][j], blk[1][j]
                acc = (a[:, None, 0] * b[None, :, 0]).astype(F32)
                for q in range(1, rank):
                    acc = (acc + (a[:, None, q] * b[None, :, q]).astype(F32)).astype(F32)
                parts.append((acc / sqrt_r).astype(F32).reshape(-1))
            else:
                parts.append(blk[j].astype(F32))
        rows.append(F32(sgn) * np.concatenate(parts))
    return np.stack(rows).astype(F32) if rows else np.zeros((0, 0), F32)


def ref_perturb(theta: np.ndarray, eps_k: np.ndarray, sigma: float) -> np.ndarray:
    """unifed_es.py:160: theta + sigma * eps[k] (two fp32 roundings)."""
    return (theta.astype(F32) + (F32(sigma) * eps_k.astype(F32)).astype(F32)).astype(F32)


# ---------------------------------------------------------------------------------------
# (3) fitness shaping (utills.py:168-178, 310-330; unifed_es.py:230-275)
# ---------------------------------------------------------------------------------------


def ref_promptnorm(S: np.ndarray, eps: float = 1e-8):
    """paper_prompt_normalized_scores (utills.py:310-330), vectorised fp32."""
    S = S.astype(F32)
    mu = S.mean(axis=0, dtype=F32)
    c = (S - mu[None, :]).astype(F32)
    sb = np.sqrt((c * c).mean(dtype=F32)).astype(F32)
    if sb < F32(eps):  # clamp_min: a NaN sigma_bar stays NaN
        sb = F32(eps)
    z = (c / sb).astype(F32)
    return z.mean(axis=1, dtype=F32), mu, sb


def ref_standardize(r: np.ndarray) -> np.ndarray:
    """standardize_fitness (utills.py:168-178): unbiased std; std<1e-8 -> zeros."""
    r = r.astype(F32)
    mean = r.mean(dtype=F32)
    with np.errstate(invalid="ignore", divide="ignore"):
        std = F32(r.std(ddof=1, dtype=F32)) if r.size > 1 else F32(np.nan)
    if std < F32(1e-8):
        return np.zeros_like(r)
    return ((r - mean) / (std + F32(1e-8))).astype(F32)


def dev_fitness(S: np.ndarray, promptnorm: bool, eps: float = 1e-8):
    """Kernel k_fitness restated in its exact sequential fp32 op order."""
    S = np.asarray(S, F32)
    n, m = S.shape
    mu = np.zeros(m, F32)
    for j in range(m):
        acc = F32(0)
        for k in range(n):
            acc = F32(acc + S[k, j])
        mu[j] = F32(acc / F32(n))
    sc = np.zeros(n, F32)
    sigma_bar = F32(np.nan)
    with np.errstate(all="ignore"):
        if promptnorm:
            ss = F32(0)
            for k in range(n):
                acc = F32(0)
                for j in range(m):
                    c = F32(S[k, j] - mu[j])
                    acc = F32(acc + F32(c * c))
                ss = F32(ss + acc)
            sb = F32(np.sqrt(F32(ss / F32(n * m))))
            if sb < F32(eps):
                sb = F32(eps)
            sigma_bar = sb
            for k in range(n):
                acc = F32(0)
                for j in range(m):
                    acc = F32(acc + F32(F32(S[k, j] - mu[j]) / sb))
                sc[k] = F32(acc / F32(m))
        else:
            for k in range(n):
                acc = F32(0)
                for j in range(m):
                    acc = F32(acc + S[k, j])
                sc[k] = F32(acc / F32(m))
        fin = np.isfinite(sc)
        nf = int(fin.sum())
        s = F32(0)
        for k in range(n):
            if fin[k]:
                s = F32(s + sc[k])
        mean = F32(s / F32(nf))
        sq = F32(0)
        for k in range(n):
            if fin[k]:
                d = F32(sc[k] - mean)
                sq = F32(sq + F32(d * d))
        std = F32(np.sqrt(F32(sq / F32(nf - 1))))
        degenerate = bool(std < F32(1e-8))
        f = np.zeros(n, F32)
        for k in range(n):
            if fin[k]:
                f[k] = F32(0) if degenerate else F32(F32(sc[k] - mean) / F32(std + F32(1e-8)))
    key = [(1, 0.0, k) if np.isnan(sc[k]) else (0, float(sc[k]), k) for k in range(n)]
    order = np.array([k for _, _, k in sorted(key)], np.int32)
    stats = np.array([sigma_bar, nf, mean, std], F32)
    return {"scores": sc, "mu": mu, "stats": stats, "fitness": f, "finite": fin.astype(np.int32),
            "order": order}


# ---------------------------------------------------------------------------------------
# (4) update + caps (utills.py:115-136, 333-349; unifed_es.py:266-281)
# ---------------------------------------------------------------------------------------


def ref_do_update(theta: np.ndarray, eps: np.ndarray, fit: np.ndarray, lr_scale: float, sigma: float):
    """EggRollNoiser.do_update: theta + (lr_scale*sigma) * mean_k(f_k eps_k)."""
    g = (fit.astype(F32)[:, None] * eps.astype(F32)).astype(F32).mean(axis=0, dtype=F32)
    return (theta.astype(F32) + (F32(lr_scale * sigma) * g).astype(F32)).astype(F32)


def ref_cap_step_norm(before: np.ndarray, after: np.ndarray, max_step_norm: float) -> np.ndarray:
    if max_step_norm is None or max_step_norm <= 0:
        return after
    d = (after - before).astype(F32)
    dn = F32(np.linalg.norm(d.astype(np.float64)))
    if dn > max_step_norm:
        after = (before + (d * F32(max_step_norm / (float(dn) + 1e-8))).astype(F32)).astype(F32)
    return after


def ref_cap_theta_norm(theta: np.ndarray, theta_max_norm: float) -> np.ndarray:
    if theta_max_norm is None or theta_max_norm <= 0:
        return theta
    n = F32(np.linalg.norm(theta.astype(np.float64)))
    if n > theta_max_norm:
        theta = (theta * F32(theta_max_norm / (float(n) + 1e-8))).astype(F32)
    return theta


def ref_es_tail(S: np.ndarray, eps: np.ndarray, theta: np.ndarray, *, promptnorm: bool, lr_scale: float,
                sigma: float, max_step_norm: float, theta_max_norm: float):
    """unifed_es.py:227-281 after S is known: scores -> finite mask -> sort -> z-score ->
    update -> caps.  Returns (theta_after, info)."""
    S = S.astype(F32)
    if promptnorm:
        scores, mu, sb = ref_promptnorm(S)
    else:
        scores, mu, sb = S.mean(axis=1, dtype=F32), S.mean(axis=0, dtype=F32), F32(np.nan)
    fin = np.isfinite(scores)
    info = {"scores": scores, "mu": mu, "sigma_bar": sb, "finite": fin}
    if not fin.any():
        info["skipped"] = True
        return theta.astype(F32), info
    info["skipped"] = False
    if fin.all():
        info["order"] = np.argsort(scores, kind="stable")
    f = ref_standardize(scores[fin])
    info["fitness"] = f
    after = ref_do_update(theta, eps[fin], f, lr_scale, sigma)
    after = ref_cap_step_norm(theta.astype(F32), after, max_step_norm)
    after = ref_cap_theta_norm(after, theta_max_norm)
    return after, info


# ---------------------------------------------------------------------------------------
# (2) PEFT LoRA linear (peft.tuners.lora.layer.Linear.forward; attached es_backend.py:193-200)
# ---------------------------------------------------------------------------------------


def ref_lora_linear(x: np.ndarray, W: np.ndarray, bias, A: np.ndarray, B: np.ndarray, scale: float) -> np.ndarray:
    """y = x W^T + bias + scale * (x A^T) B^T, evaluated in fp64 (dropout = 0 at unifed_es.py:390)."""
    x64 = x.astype(np.float64)
    y = x64 @ W.astype(np.float64).T
    if bias is not None:
        y = y + bias.astype(np.float64)[None, :]
    return y + scale * ((x64 @ A.astype(np.float64).T) @ B.astype(np.float64).T)


def ref_lora_linear_pop(x: np.ndarray, W: np.ndarray, bias, theta_pop: np.ndarray, offA: int, offB: int,
                        r: int, scale: float, rows_per_member: int) -> np.ndarray:
    """Members stacked along rows; member k uses theta_pop[k] slices (unflatten_to_params)."""
    M, K = x.shape
    N = W.shape[0]
    out = np.empty((M, N), np.float64)
    for k in range(-(-M // rows_per_member)):
        sl = slice(k * rows_per_member, min(M, (k + 1) * rows_per_member))
        A = theta_pop[k, offA:offA + r * K].reshape(r, K)
        B = theta_pop[k, offB:offB + N * r].reshape(N, r)
        out[sl] = ref_lora_linear(x[sl], W, bias, A, B, scale)
    return out
