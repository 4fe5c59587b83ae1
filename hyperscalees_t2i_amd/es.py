"""Host mirror of the reference's ES utilities (`utills.py`), backed by libeggroll kernels.

Same names, argument meaning and return values as amit154154/HyperscaleES_T2I `utills.py`, so
`from hyperscalees_t2i_amd.es import *` can replace the reference's `from utills import *` on the
ES hot path.  Differences are deliberate and documented per function:
  * noise is counter-based (Philox keyed by an explicit seed) instead of torch's global RNG —
    bit-exact reproduction of torch.randn streams is impossible across RNGs;
    feeding reference factors through `eps_from_factors` reproduces the reference eps exactly;
  * the engine path never materialises eps [pop, D] and, by default, never stores the factors
    either: `EggRollNoiser.epoch_noise` returns a `SeededFactors` handle (the epoch seed), and the
    perturb / update kernels regenerate every factor value where they consume it
    (`EggRollNoiser.perturb`, `EggRollNoiser.update_from_factors`); a factor TENSOR (`sample_factors`,
    or reference factors injected for parity tests) runs the same kernels on the stored values —
    both give the same bits.
"""
from __future__ import annotations

from typing import List, Optional, Sequence, Tuple, Union

import numpy as np
import torch
from torch import nn

from . import kernels as K
from .kernels import ThetaLayout, n_base_samples


class SeededFactors:
    """The factors of one epoch, held as the Philox key that generates them (no buffer): base sample j's
    factor element g is Philox4x32-10(counter (g / 4, j, tag), key seed) -> Box-Muller, as the noise
    kernel writes it (include/eggroll.h)."""

    def __init__(self, seed: int, n_base: int):
        self.seed, self.n_base = int(seed), int(n_base)

    def materialise(self, layout: ThetaLayout, device) -> torch.Tensor:
        """The stored form [n_base, factor_ld] (eggroll_noise_factors) — for tests and eps materialisation."""
        return K.noise_factors(self.seed, self.n_base, layout, device)


Factors = Union[torch.Tensor, SeededFactors]


class EggRollNoiser:
    """Low-rank EGGROLL noise E = a b^T / sqrt(r) per parameter matrix (utills.py:14-136)."""

    def __init__(self, param_shapes, sigma: float, lr_scale: float, rank: int = 1, use_antithetic: bool = False):
        self.param_shapes = list(param_shapes)
        self.sigma = sigma
        self.lr_scale = lr_scale
        self.rank = rank
        self.use_antithetic = use_antithetic
        self.layout = ThetaLayout([tuple(s) for s in self.param_shapes], rank)
        self.num_params = int(self.layout.D)  # utills.py:41
        self._ws = {}

    # ---- factor form (engine path) -------------------------------------------------
    def n_base(self, pop_size: int) -> int:
        return n_base_samples(pop_size, self.use_antithetic)

    def sample_factors(self, pop_size: int, device, seed: Optional[int] = None) -> torch.Tensor:
        """All base samples' factors [n_base, factor_ld] fp32 (noise kernel).  seed=None draws a
        seed from torch's global generator, so torch.manual_seed(epoch) makes it reproducible
        exactly where the reference relied on it (unifed_es.py:120-122)."""
        if seed is None:
            seed = int(torch.randint(0, 2 ** 62, (1,)).item())
        return K.noise_factors(seed, self.n_base(pop_size), self.layout, device)

    def epoch_noise(self, pop_size: int, seed: Optional[int] = None) -> SeededFactors:
        """The epoch's factors as a seed handle (the engine path: regenerated inside perturb / update).
        seed=None draws one from torch's global generator, as sample_factors does."""
        if seed is None:
            seed = int(torch.randint(0, 2 ** 62, (1,)).item())
        return SeededFactors(seed, self.n_base(pop_size))

    def perturb(self, theta: Optional[torch.Tensor], factors: Factors, pop_size: int, member_lo: int, member_hi: int,
                out: Optional[torch.Tensor] = None, device=None) -> torch.Tensor:
        """theta_k = theta + sigma * eps_k for members [lo, hi)  (unifed_es.py:160)."""
        if isinstance(factors, SeededFactors):
            dev = theta.device if theta is not None else (out.device if out is not None else device)
            return K.perturb_seeded(theta, factors.seed, self.layout, pop_size, self.use_antithetic, member_lo,
                                    member_hi, self.sigma, dev, out=out)
        return K.perturb(theta, factors, self.layout, pop_size, self.use_antithetic, member_lo, member_hi,
                         self.sigma, out=out)

    def eps_from_factors(self, factors: Factors, pop_size: int, device=None) -> torch.Tensor:
        """Materialised eps [pop, D] in the reference layout (utills.py:70-106)."""
        if isinstance(factors, SeededFactors):
            return K.perturb_seeded(None, factors.seed, self.layout, pop_size, self.use_antithetic, 0, pop_size, 1.0,
                                    device)
        return K.perturb(None, factors, self.layout, pop_size, self.use_antithetic, 0, pop_size, 1.0)

    def update_from_factors(self, theta: torch.Tensor, factors: Factors, fit: dict, pop_size: int,
                            max_step_norm: float = 0.0, theta_max_norm: float = 0.0,
                            out: Optional[torch.Tensor] = None) -> torch.Tensor:
        """do_update + cap_step_norm + cap_theta_norm fused (utills.py:115-136, 333-349)."""
        ws = self._ws.get(theta.device)
        if ws is None:
            ws = self._ws[theta.device] = K.UpdateWorkspace(self.layout, theta.device)
        lr = float(self.lr_scale * self.sigma)
        if isinstance(factors, SeededFactors):
            return K.update_seeded(theta, factors.seed, fit, self.layout, pop_size, self.use_antithetic, lr,
                                   max_step_norm, theta_max_norm, out=out, workspace=ws)
        return K.update(theta, factors, fit, self.layout, pop_size, self.use_antithetic, lr, max_step_norm,
                        theta_max_norm, out=out, workspace=ws)

    # ---- reference API -------------------------------------------------------------
    def sample_eps(self, pop_size: int, device, seed: Optional[int] = None) -> torch.Tensor:
        """utills.py:70-106: eps [pop, D] with the antithetic layout."""
        return self.eps_from_factors(self.sample_factors(pop_size, device, seed), pop_size)

    def convert_fitnesses(self, raw_scores: torch.Tensor) -> torch.Tensor:
        """utills.py:108-113."""
        return standardize_fitness(raw_scores)

    def do_update(self, theta: torch.Tensor, eps: torch.Tensor, fitnesses: torch.Tensor) -> torch.Tensor:
        """utills.py:115-136 on a materialised eps (compat form; the engine uses update_from_factors)."""
        lr = self.lr_scale * self.sigma
        grad_est = (fitnesses.unsqueeze(1) * eps).mean(dim=0)
        return theta + lr * grad_est


# ---------------------------------------------------------------------------------------
# trainable-parameter plumbing (utills.py:141-162)
# ---------------------------------------------------------------------------------------


def get_trainable_params_and_shapes(module: nn.Module):
    params, shapes = [], []
    for p in module.parameters():
        if p.requires_grad:
            params.append(p)
            shapes.append(p.shape)
    return params, shapes


def flatten_params(params):
    return torch.cat([p.data.view(-1) for p in params])


def unflatten_to_params(flat: torch.Tensor, params, shapes):
    assert flat.numel() == sum(p.numel() for p in params)
    idx = 0
    for p, shape in zip(params, shapes):
        numel = p.numel()
        p.data.copy_(flat[idx: idx + numel].view(shape))
        idx += numel


# ---------------------------------------------------------------------------------------
# fitness shaping (utills.py:168-178, 310-349) — kernel (3)
# ---------------------------------------------------------------------------------------


def standardize_fitness(rewards: torch.Tensor) -> torch.Tensor:
    """(r - mean) / (std + 1e-8), unbiased std, zeros if std < 1e-8 (utills.py:168-178).
    The reference only calls it on finite scores (unifed_es.py:275); a non-finite input gives
    all-NaN like the reference."""
    r = rewards.detach().float().contiguous()
    if not bool(torch.isfinite(r).all()):
        return torch.full_like(r, float("nan"))
    return K.fitness(r.view(-1, 1), promptnorm=False)["fitness"].view_as(r)


def paper_prompt_normalized_scores(S: torch.Tensor, eps: float = 1e-8):
    """utills.py:310-330: scores [n], mu_q [m], sigma_bar (scalar tensor)."""
    if S.ndim != 2:
        raise ValueError(f"S must be [n, m], got {tuple(S.shape)}")
    out = K.fitness(S.float().contiguous(), promptnorm=True, eps=float(eps))
    return out["scores"], out["mu"], out["stats"][0]


def cap_theta_norm(theta: torch.Tensor, theta_max_norm: float) -> torch.Tensor:
    """utills.py:333-339 (compat form; the engine fuses it into the update kernel)."""
    if theta_max_norm is None or theta_max_norm <= 0:
        return theta
    n = theta.norm()
    if n > theta_max_norm:
        theta = theta * (theta_max_norm / (n + 1e-8))
    return theta


def cap_step_norm(theta_before: torch.Tensor, theta_after: torch.Tensor, max_step_norm: float) -> torch.Tensor:
    """utills.py:342-349 (compat form)."""
    if max_step_norm is None or max_step_norm <= 0:
        return theta_after
    d = theta_after - theta_before
    dn = d.norm()
    if dn > max_step_norm:
        theta_after = theta_before + d * (max_step_norm / (dn + 1e-8))
    return theta_after


# ---------------------------------------------------------------------------------------
# prompt/class sampling (utills.py:364-379) — exact integer host logic
# ---------------------------------------------------------------------------------------


def sample_indices_unique(seed: int, total: int, k: int) -> List[int]:
    if total <= 0:
        raise ValueError("total must be >= 1")
    if k <= 0:
        raise ValueError("k must be >= 1")
    rng = np.random.RandomState(int(seed))
    if k >= total:
        return list(range(total))
    idx = rng.choice(np.arange(total, dtype=np.int64), size=k, replace=False)
    return idx.tolist()


def sample_classes_unique(seed: int, allowed_classes="all", classes_per_gen: int = 4,
                          num_classes_total: int = 1000) -> List[int]:
    """VarBackend._sample_classes_unique (es_backend.py:377-396): class ids for one epoch, drawn
    without replacement by np.random.RandomState(seed).choice from the allowed pool."""
    rng = np.random.RandomState(int(seed))
    if allowed_classes is None or allowed_classes == "all":
        pool = np.arange(num_classes_total, dtype=np.int64)
    else:
        pool = np.unique(np.array(list(allowed_classes), dtype=np.int64))
        pool = pool[(pool >= 0) & (pool < num_classes_total)]
        if pool.size == 0:
            pool = np.arange(num_classes_total, dtype=np.int64)
    m = int(classes_per_gen)
    if m <= 0:
        raise ValueError("classes_per_gen must be >= 1")
    if m > pool.size:
        raise ValueError(f"classes_per_gen ({m}) > pool size ({pool.size})")
    return rng.choice(pool, size=m, replace=False).tolist()


def repeat_batches(ids_unique: List[int], repeats: int) -> List[int]:
    if repeats <= 0:
        raise ValueError("repeats must be >= 1")
    return [i for _ in range(repeats) for i in ids_unique]


def parse_int_list(s: str) -> Union[str, List[int]]:
    s = (s or "").strip()
    if s.lower() == "all" or s == "":
        return "all"
    return [int(x.strip()) for x in s.split(",") if x.strip() != ""]
