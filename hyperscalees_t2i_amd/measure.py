"""Live roofline measurement of the HBM-bound ES kernels (noise, perturb, fitness, update).

Used by bench.py and tools/aux_probe.py.  Each kernel is timed with HIP events recorded on the
stream it is launched on (torch's current stream — every libeggroll wrapper launches there) and
priced against its ALGORITHMIC bytes:
  noise_factors  4 * n_base * F                       (factors written once)
  perturb        4 * (n_local * D + D + n_used * F)    (theta_pop written, theta + the local members'
                                                       factor sets read)
  update         4 * (n_base * F + 2 * D)              (factors + theta read, theta' written)
  perturb_seeded 4 * (n_local * D + D)                 (factors regenerated in the kernel: no factor bytes)
  update_seeded  4 * (2 * D)                           (idem)
The seeded kernels replace HBM bytes by Philox4x32-10 + Box-Muller work: `philox_quads` per launch
(one quad = 4 normals; perturb regenerates each local member's long factors, update every base
sample's) is reported next to the byte-based fraction.
with F = layout.factor_len_packed, the useful factor values per base sample (the 16-byte alignment
pads of the device layout, < 0.2 % at the Sana shapes, are not counted).
The fitness kernel reads a [pop, m] score matrix: latency-bound, reported in microseconds.
"""
from __future__ import annotations

from typing import Dict, Optional

import torch

from . import kernels as K
from .kernels import ThetaLayout, n_base_samples

HBM_PEAK_GBPS = 8000.0  # MI355X HBM3E (MI355X_MICROARCH.md)


def _time(fn, it: int = 20) -> float:
    """Average seconds per call over `it` back-to-back launches (one warm-up call first).

    The launches are queued behind a ~2 ms spin kernel, so the GPU runs them back to back: the
    average is the kernels' own duration (plus the dispatch gap), which is what rocprof reports —
    not the host's ctypes/Python launch rate, which exceeds a 5-20 us kernel."""
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda._sleep(5_000_000)
    s.record()
    for _ in range(it):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / it * 1e-3


def _entry(sec: float, byt: float) -> Dict[str, float]:
    gbps = byt / sec / 1e9
    return {"us": sec * 1e6, "bytes": byt, "GBps": gbps, "frac": gbps / HBM_PEAK_GBPS}


def used_bases(pop: int, antithetic: bool, member_lo: int, member_hi: int) -> int:
    """Distinct base samples the members [lo, hi) read (reference antithetic layout utills.py:88-105)."""
    h = pop // 2
    js = set()
    for k in range(member_lo, member_hi):
        if not antithetic:
            js.add(k)
        else:
            js.add(k if k < h else (k - h if k < 2 * h else h))
    return len(js)


def aux_kernel_rooflines(layout: ThetaLayout, pop: int, member_lo: int, member_hi: int, device,
                         sigma: float = 1e-2, lr: float = 1e-3, theta: Optional[torch.Tensor] = None,
                         antithetic: bool = True, m: int = 4, it: int = 20) -> Dict[str, Dict[str, float]]:
    device = torch.device(device)
    nb = n_base_samples(pop, antithetic)
    nl = member_hi - member_lo
    D = layout.D
    if theta is None:
        theta = torch.randn(D, device=device) * 0.01
    out: Dict[str, Dict[str, float]] = {}
    fac = K.noise_factors(0, nb, layout, device)
    sec = _time(lambda: K.noise_factors(0, nb, layout, device, out=fac), it)
    F = layout.factor_len_packed
    out["noise_factors"] = _entry(sec, 4.0 * nb * F)
    tp = torch.empty((nl, D), dtype=torch.float32, device=device)
    sec = _time(lambda: K.perturb(theta, fac, layout, pop, antithetic, member_lo, member_hi, sigma, out=tp), it)
    nu = used_bases(pop, antithetic, member_lo, member_hi)
    out["perturb"] = _entry(sec, 4.0 * (nl * D + D + nu * F))
    S = torch.randn(pop, m, device=device) + 21
    fit = K.fitness(S, True)
    sec = _time(lambda: K.fitness(S, True), it)
    out["fitness"] = {"us": sec * 1e6, "note": f"latency-bound single workgroup ({pop}x{m} input)"}
    ws = K.UpdateWorkspace(layout, device)
    newt = torch.empty_like(theta)
    sec = _time(lambda: K.update(theta, fac, fit, layout, pop, antithetic, lr, 0.0, 40.0, out=newt, workspace=ws), it)
    out["update"] = _entry(sec, 4.0 * (nb * F + 2 * D))
    out["update"]["note"] = "update kernel + the caps pass (theta_max_norm 40): two dependent launches"
    # the same update without caps: one launch (k_update only), i.e. the HBM-bound kernel by itself
    sec = _time(lambda: K.update(theta, fac, fit, layout, pop, antithetic, lr, 0.0, 0.0, out=newt, workspace=ws), it)
    out["update_nocaps"] = _entry(sec, 4.0 * (nb * F + 2 * D))
    out["update_nocaps"]["note"] = "the update kernel alone (no caps): the HBM-bound launch"
    out["update_caps_pass"] = {"us": max(out["update"]["us"] - out["update_nocaps"]["us"], 0.0),
                               "note": "the caps pass: a fixed-order reduction of n_tiles x 32 B of norm partials "
                                       "plus one dependent launch; latency-bound (rescales only if a cap fires)"}
    # the engine path: factors regenerated inside perturb / update (no noise launch, no factor bytes)
    sf = K.perturb_seeded
    sec = _time(lambda: sf(theta, 0, layout, pop, antithetic, member_lo, member_hi, sigma, device, out=tp), it)
    out["perturb_seeded"] = _entry(sec, 4.0 * (nl * D + D))
    out["perturb_seeded"]["philox_quads"] = nl * F / 4.0
    sec = _time(lambda: K.update_seeded(theta, 0, fit, layout, pop, antithetic, lr, 0.0, 40.0, out=newt, workspace=ws),
                it)
    out["update_seeded"] = _entry(sec, 4.0 * 2 * D)
    out["update_seeded"]["philox_quads"] = nb * F / 4.0
    sec = _time(lambda: K.update_seeded(theta, 0, fit, layout, pop, antithetic, lr, 0.0, 0.0, out=newt, workspace=ws),
                it)
    out["update_seeded_nocaps"] = _entry(sec, 4.0 * 2 * D)
    out["update_seeded_nocaps"]["philox_quads"] = nb * F / 4.0
    out["es_epoch_us"] = {
        "stored": out["noise_factors"]["us"] + out["perturb"]["us"] + out["update"]["us"],
        "seeded": out["perturb_seeded"]["us"] + out["update_seeded"]["us"],
        "note": "noise + perturb + update(+caps) with the factors stored in HBM vs regenerated inside perturb / "
                "update (the engine default); fitness and the all-gather are the same in both"}
    # empirical write / copy floors on this box for the same byte counts (torch's fill and copy kernels):
    # the noise kernel writes nb * F floats and also runs Philox4x32-10 + Box-Muller per 4 of them, so it is
    # priced against both the HBM peak (frac) and the plain-store floor (frac_of_store_floor)
    sec_fill = _time(lambda: fac.zero_(), it)
    fill_gbps = 4.0 * nb * layout.factor_ld / sec_fill / 1e9
    out["noise_factors"]["store_floor_GBps"] = fill_gbps
    out["noise_factors"]["frac_of_store_floor"] = out["noise_factors"]["GBps"] / fill_gbps
    out["sizes"] = {"pop": pop, "members": [member_lo, member_hi], "n_base": nb, "D": D,
                    "factor_len": F, "n_tiles": layout.n_tiles}
    return out


def achievable_peaks(device) -> Dict[str, float]:
    """the bf16 GEMM peak measured on this box next to the vendor figure — hipBLASLt's and
    libeggroll's plain GEMM at a large shape (16384 x 8192 x 8192).  Outside the timed region."""
    g = torch.Generator(device=device).manual_seed(0)
    M = N = 8192
    Kd = 8192
    x = torch.randn(2 * M, Kd, device=device, generator=g).bfloat16()
    w = (torch.randn(N, Kd, device=device, generator=g) * Kd ** -0.5).bfloat16()
    fl = 2.0 * 2 * M * N * Kd
    t_hip = _time(lambda: torch.nn.functional.linear(x, w), it=10)
    out = torch.empty(2 * M, N, device=device, dtype=torch.bfloat16)
    t_egg = _time(lambda: K.lora_linear_pop(x, w, None, None, 0, 0, 0, 0.0, 2 * M, out=out), it=10)
    del x, w, out
    torch.cuda.empty_cache()
    return {"bf16_gemm_tflops_hipblaslt": fl / t_hip / 1e12, "bf16_gemm_tflops_eggroll": fl / t_egg / 1e12,
            "note": "16384x8192x8192 bf16 GEMM, average of 10 launches (HIP events); the HBM side has no library "
                    "kernel faster than libeggroll's own ES kernels to calibrate against (torch's 4 GiB copy: 4.7 TB/s)"}
