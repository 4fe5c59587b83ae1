"""Torch-tensor front end of the libeggroll C-ABI (device memory + streams come from PyTorch).

Every function here launches HIP kernels through include/eggroll.h on the tensor's device and
the current torch stream; none of them computes anything on the host.  Tensors must live on
a ROCm device (`cuda:*` in torch) — a CPU tensor raises.
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np
import torch

from . import _lib

CHUNK = 1024  # EGGROLL_CHUNK in include/eggroll.h


def _dev(t: torch.Tensor, what: str, dtype=None, contiguous: bool = True) -> torch.Tensor:
    if not isinstance(t, torch.Tensor) or t.device.type != "cuda":
        raise _lib.EggrollError(f"{what}: expected a ROCm device tensor, got "
                                f"{getattr(t, 'device', type(t))} (no CPU fallback)")
    if dtype is not None and t.dtype != dtype:
        raise _lib.EggrollError(f"{what}: expected dtype {dtype}, got {t.dtype}")
    if contiguous and not t.is_contiguous():
        raise _lib.EggrollError(f"{what}: tensor must be contiguous")
    return t


def _p(t: Optional[torch.Tensor]):
    return None if t is None else t.data_ptr()


def _stream(device: torch.device):
    return torch.cuda.current_stream(device).cuda_stream


# ---------------------------------------------------------------------------------------
# theta layout (reference utills.py:141-162: concat of trainable params, row-major)
# ---------------------------------------------------------------------------------------


def _pad4(x: int) -> int:
    return -(-x // 4) * 4


@dataclass
class ThetaLayout:
    """Per-parameter records of the flat theta vector and of one base sample's factors.

    Factor layout (include/eggroll.h): per matrix a [rows][r] then b [cols][r], each segment padded
    to a multiple of 4 floats so every segment is 16-byte aligned; 1-D params: numel values (padded).
    The reference's contiguous order (torch.cat of the randn blocks, utills.py:59-66) is the same
    sequence without the pads: `pack_factors` / `unpack_factors` convert."""

    shapes: List[Tuple[int, ...]]
    rank: int
    mats: np.ndarray = field(init=False)      # [n_mats, 6] int64 (eggroll_mat_t)
    D: int = field(init=False)
    factor_len: int = field(init=False)       # padded length the noise kernel fills
    factor_len_packed: int = field(init=False)  # useful factor values per base sample (no pads)
    factor_ld: int = field(init=False)        # row stride of factor buffers (multiple of 4)
    total_chunks: int = field(init=False)
    theta_offsets: List[int] = field(init=False)

    def __post_init__(self):
        self.shapes = [tuple(int(x) for x in s) for s in self.shapes]
        if self.rank < 1:
            raise ValueError("egg rank must be >= 1")
        recs, offs, segs = [], [], []
        toff = foff = coff = packed = 0
        for s in self.shapes:
            if len(s) == 2:
                m, n = s
                numel = m * n
                seg = [(foff, m * self.rank), (foff + _pad4(m * self.rank), n * self.rank)]
                fl = _pad4(m * self.rank) + _pad4(n * self.rank)
            else:
                m, n = int(np.prod(s)), 0
                numel = m
                seg = [(foff, m)]
                fl = _pad4(m)
            recs.append((m, n, toff, foff, coff, 0))
            offs.append(toff)
            segs.extend(seg)
            packed += sum(ln for _, ln in seg)
            toff += numel
            foff += fl
            coff += -(-numel // CHUNK)
        self.mats = np.array(recs, dtype=np.int64).reshape(-1, 6)
        self.D, self.factor_len, self.total_chunks = toff, foff, coff
        self.factor_len_packed = packed
        self.factor_ld = _pad4(foff)
        self.theta_offsets = offs
        self._segments = segs
        self._dev_cache: Dict[str, torch.Tensor] = {}
        self._tiles: Optional[np.ndarray] = None

    @property
    def n_mats(self) -> int:
        return len(self.shapes)

    def mats_on(self, device) -> torch.Tensor:
        key = str(torch.device(device))
        t = self._dev_cache.get(key)
        if t is None:
            t = torch.from_numpy(self.mats.copy()).to(device)
            self._dev_cache[key] = t
        return t

    def tile_table(self) -> np.ndarray:
        """[n_tiles, 2] int32 (eggroll_tile_t) from the library's host builder eggroll_tile_table."""
        if self._tiles is None:
            lib = _lib.load()
            mats = np.ascontiguousarray(self.mats)
            n = int(lib.eggroll_tile_table(mats.ctypes.data, self.n_mats, self.rank, None, 0))
            if n < 1:
                raise _lib.EggrollError(f"eggroll_tile_table failed ({n}): {lib.eggroll_last_error().decode()}")
            tiles = np.zeros((n, 2), dtype=np.int32)
            got = int(lib.eggroll_tile_table(mats.ctypes.data, self.n_mats, self.rank, tiles.ctypes.data, n))
            if got != n:
                raise _lib.EggrollError("eggroll_tile_table: size changed between calls")
            self._tiles = tiles
        return self._tiles

    @property
    def n_tiles(self) -> int:
        return int(self.tile_table().shape[0])

    def tiles_on(self, device) -> torch.Tensor:
        key = "tiles:" + str(torch.device(device))
        t = self._dev_cache.get(key)
        if t is None:
            t = torch.from_numpy(self.tile_table().copy()).to(device)
            self._dev_cache[key] = t
        return t

    def pack_factors(self, contig) -> np.ndarray:
        """Reference-order factors [p, factor_len_packed] -> this layout [p, factor_ld] (pads = 0)."""
        contig = np.asarray(contig, dtype=np.float32)
        out = np.zeros((contig.shape[0], self.factor_ld), np.float32)
        src = 0
        for off, ln in self._segments:
            out[:, off:off + ln] = contig[:, src:src + ln]
            src += ln
        return out

    def unpack_factors(self, padded) -> np.ndarray:
        """This layout [p, >= factor_len] -> the reference's contiguous order [p, factor_len_packed]."""
        padded = np.asarray(padded, dtype=np.float32)
        return np.concatenate([padded[:, off:off + ln] for off, ln in self._segments], axis=1)


def n_base_samples(pop: int, antithetic: bool) -> int:
    """reference utills.py:88-89"""
    return (pop // 2 + pop % 2) if antithetic else pop


# ---------------------------------------------------------------------------------------
# (1) noise factors
# ---------------------------------------------------------------------------------------


def noise_factors(seed: int, n_base: int, layout: ThetaLayout, device, base_lo: int = 0,
                  out: Optional[torch.Tensor] = None) -> torch.Tensor:
    device = torch.device(device)
    rows = n_base - base_lo
    if out is None:
        out = torch.empty((rows, layout.factor_ld), dtype=torch.float32, device=device)
    _dev(out, "noise_factors(out)", torch.float32)
    _lib.call("eggroll_noise_factors", int(seed) & 0xFFFFFFFFFFFFFFFF, base_lo, n_base, layout.factor_len,
              layout.factor_ld, out.data_ptr(), _stream(device))
    return out


def philox_words(seed: int, j: int, n_quads: int, device) -> torch.Tensor:
    out = torch.empty(4 * n_quads, dtype=torch.int32, device=device)
    _lib.call("eggroll_philox_words", int(seed), int(j), int(n_quads), out.data_ptr(), _stream(out.device))
    return out


def perturb(theta: Optional[torch.Tensor], factors: torch.Tensor, layout: ThetaLayout, pop: int, antithetic: bool,
            member_lo: int, member_hi: int, sigma: float, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """theta_k = theta + sigma * eps_k for k in [member_lo, member_hi) (theta=None: eps rows)."""
    _dev(factors, "perturb(factors)", torch.float32)
    device = factors.device
    if theta is not None:
        _dev(theta, "perturb(theta)", torch.float32)
    n = member_hi - member_lo
    if out is None:  # rows padded to a multiple of 4 floats: 16-byte aligned rows take the vector path
        out = torch.empty((n, _pad4(layout.D)), dtype=torch.float32, device=device)[:, :layout.D]
    if out.dim() != 2 or out.stride(1) != 1 or out.shape[1] < layout.D:
        raise _lib.EggrollError("perturb(out): expected a [n, >= D] fp32 device tensor with unit inner stride")
    if out.device.type != "cuda" or out.dtype != torch.float32:
        raise _lib.EggrollError("perturb(out): expected a ROCm fp32 tensor (no CPU fallback)")
    _lib.call("eggroll_perturb", _p(theta), factors.data_ptr(), factors.stride(0), factors.shape[0],
              layout.mats_on(device).data_ptr(), layout.tiles_on(device).data_ptr(), layout.n_tiles, layout.D,
              layout.rank, pop, int(bool(antithetic)), member_lo, member_hi, float(sigma), out.data_ptr(),
              out.stride(0), _stream(device))
    return out


def perturb_seeded(theta: Optional[torch.Tensor], seed: int, layout: ThetaLayout, pop: int, antithetic: bool,
                   member_lo: int, member_hi: int, sigma: float, device, out: Optional[torch.Tensor] = None
                   ) -> torch.Tensor:
    """perturb() with the factors regenerated in the kernel from `seed` (eggroll_perturb_seeded): bit-identical
    to perturb(theta, noise_factors(seed, n_base), ...) with no factor buffer."""
    device = torch.device(device)
    if theta is not None:
        _dev(theta, "perturb_seeded(theta)", torch.float32)
    n = member_hi - member_lo
    if out is None:
        out = torch.empty((n, _pad4(layout.D)), dtype=torch.float32, device=device)[:, :layout.D]
    if out.dim() != 2 or out.stride(1) != 1 or out.shape[1] < layout.D:
        raise _lib.EggrollError("perturb_seeded(out): expected a [n, >= D] fp32 device tensor with unit inner stride")
    if out.device.type != "cuda" or out.dtype != torch.float32:
        raise _lib.EggrollError("perturb_seeded(out): expected a ROCm fp32 tensor (no CPU fallback)")
    _lib.call("eggroll_perturb_seeded", int(seed) & 0xFFFFFFFFFFFFFFFF, _p(theta), layout.mats_on(device).data_ptr(),
              layout.tiles_on(device).data_ptr(), layout.n_tiles, layout.D, layout.rank, pop, int(bool(antithetic)),
              member_lo, member_hi, float(sigma), out.data_ptr(), out.stride(0), _stream(device))
    return out


# ---------------------------------------------------------------------------------------
# (3) fitness
# ---------------------------------------------------------------------------------------


def fitness(S: torch.Tensor, promptnorm: bool, eps: float = 1e-8) -> Dict[str, torch.Tensor]:
    """scores/mu/stats/fitness/finite/order of S [n, m] (see include/eggroll.h); eps = the
    promptnorm sigma_bar clamp (utills.py:310)."""
    _dev(S, "fitness(S)", torch.float32)
    if S.ndim != 2:
        raise ValueError(f"S must be [n, m], got {tuple(S.shape)}")
    n, m = S.shape
    dev = S.device
    out = {
        "scores": torch.empty(n, dtype=torch.float32, device=dev),
        "mu": torch.empty(m, dtype=torch.float32, device=dev),
        "stats": torch.empty(4, dtype=torch.float32, device=dev),
        "fitness": torch.empty(n, dtype=torch.float32, device=dev),
        "finite": torch.empty(n, dtype=torch.int32, device=dev),
        "order": torch.empty(n, dtype=torch.int32, device=dev),
    }
    _lib.call("eggroll_fitness", S.data_ptr(), n, m, int(bool(promptnorm)), float(eps), out["scores"].data_ptr(),
              out["mu"].data_ptr(), out["stats"].data_ptr(), out["fitness"].data_ptr(), out["finite"].data_ptr(),
              out["order"].data_ptr(), _stream(dev))
    return out


# ---------------------------------------------------------------------------------------
# (4) update
# ---------------------------------------------------------------------------------------


class UpdateWorkspace:
    def __init__(self, layout: ThetaLayout, device):
        nbytes = int(_lib.load().eggroll_update_workspace_bytes(layout.n_tiles))
        self.buf = torch.zeros(-(-nbytes // 16) * 16, dtype=torch.uint8, device=device)  # done counter starts at 0


def update(theta: torch.Tensor, factors: torch.Tensor, fit: Dict[str, torch.Tensor], layout: ThetaLayout, pop: int,
           antithetic: bool, lr: float, max_step_norm: float, theta_max_norm: float,
           out: Optional[torch.Tensor] = None, workspace: Optional[UpdateWorkspace] = None) -> torch.Tensor:
    """theta' = caps(theta + lr * mean_k f_k eps_k) with lr = lr_scale * sigma (utills.py:131)."""
    _dev(theta, "update(theta)", torch.float32)
    _dev(factors, "update(factors)", torch.float32)
    dev = theta.device
    if out is None:
        out = torch.empty_like(theta)
    if workspace is None:
        workspace = UpdateWorkspace(layout, dev)
    _lib.call("eggroll_update", theta.data_ptr(), factors.data_ptr(), factors.stride(0), factors.shape[0],
              fit["fitness"].data_ptr(), fit["stats"].data_ptr(), pop, int(bool(antithetic)),
              layout.mats_on(dev).data_ptr(), layout.tiles_on(dev).data_ptr(), layout.n_tiles, layout.D, layout.rank,
              float(lr),
              float(max_step_norm or 0.0), float(theta_max_norm or 0.0), workspace.buf.data_ptr(), out.data_ptr(),
              _stream(dev))
    return out


def update_seeded(theta: torch.Tensor, seed: int, fit: Dict[str, torch.Tensor], layout: ThetaLayout, pop: int,
                  antithetic: bool, lr: float, max_step_norm: float, theta_max_norm: float,
                  out: Optional[torch.Tensor] = None, workspace: Optional[UpdateWorkspace] = None) -> torch.Tensor:
    """update() with the factors regenerated in the kernel from `seed` (eggroll_update_seeded)."""
    _dev(theta, "update_seeded(theta)", torch.float32)
    dev = theta.device
    if out is None:
        out = torch.empty_like(theta)
    if workspace is None:
        workspace = UpdateWorkspace(layout, dev)
    _lib.call("eggroll_update_seeded", int(seed) & 0xFFFFFFFFFFFFFFFF, theta.data_ptr(), fit["fitness"].data_ptr(),
              fit["stats"].data_ptr(), pop, int(bool(antithetic)), layout.mats_on(dev).data_ptr(),
              layout.tiles_on(dev).data_ptr(), layout.n_tiles, layout.D, layout.rank, float(lr),
              float(max_step_norm or 0.0), float(theta_max_norm or 0.0), workspace.buf.data_ptr(), out.data_ptr(),
              _stream(dev))
    return out


# ---------------------------------------------------------------------------------------
# (2) population LoRA linear
# ---------------------------------------------------------------------------------------


def lora_linear_pop(x: torch.Tensor, W: torch.Tensor, bias: Optional[torch.Tensor], theta_pop: Optional[torch.Tensor],
                    offA: int, offB: int, r: int, scale: float, rows_per_member: int,
                    out: Optional[torch.Tensor] = None, T_ws: Optional[torch.Tensor] = None,
                    kernel: int = 0) -> torch.Tensor:
    """Y = x W^T + bias + scale * (x A_k^T) B_k^T with member k = row // rows_per_member.

    x: [M, K] bf16; W: [N, K] bf16; bias: [N] bf16 or None; theta_pop: [n_members, ld] fp32.
    r = 0 runs the plain base GEMM (no LoRA term).  kernel: 0 = automatic choice, else an explicit
    kernel for A/B measurement (eggroll_lora_linear_pop_sel)."""
    _dev(x, "lora_linear_pop(x)", torch.bfloat16)
    _dev(W, "lora_linear_pop(W)", torch.bfloat16)
    M, K = x.shape
    N = W.shape[0]
    if W.shape[1] != K:
        raise ValueError(f"W {tuple(W.shape)} does not match x {tuple(x.shape)}")
    if bias is not None:
        _dev(bias, "lora_linear_pop(bias)", torch.bfloat16)
    if out is None:
        out = torch.empty((M, N), dtype=torch.bfloat16, device=x.device)
    if r > 0:
        _dev(theta_pop, "lora_linear_pop(theta_pop)", torch.float32)
        n_members = -(-M // rows_per_member)
        if theta_pop.shape[0] < n_members:
            raise ValueError(f"theta_pop has {theta_pop.shape[0]} members, rows need {n_members}")
        need = lora_workspace_numel(M, K, r, rows_per_member)
        if T_ws is None or T_ws.numel() < need:
            T_ws = torch.empty(need, dtype=torch.float32, device=x.device)
        ld_t = theta_pop.stride(0)
    else:
        ld_t = 0
    _lib.call("eggroll_lora_linear_pop_sel", x.data_ptr(), x.stride(0), W.data_ptr(), W.stride(0), _p(bias),
              _p(theta_pop) if r > 0 else None, ld_t, offA, offB, r, float(scale), rows_per_member, M, N, K,
              out.data_ptr(), out.stride(0), _p(T_ws) if r > 0 else None, int(kernel), _stream(x.device))
    return out


EPI = {None: 0, "silu": 1, "res": 2, "gated": 3, "res32": 4, "gated32": 5, "gelu": 6, "mul": 7, "gelu_erf": 8}


def lora_linear_pop_epi(x: torch.Tensor, W: torch.Tensor, bias: Optional[torch.Tensor], theta_pop: Optional[torch.Tensor],
                        offA: int, offB: int, r: int, scale: float, rows_per_member: int, epi: str,
                        res: Optional[torch.Tensor] = None, gate: Optional[torch.Tensor] = None,
                        rows_per_group: int = 1, out: Optional[torch.Tensor] = None,
                        T_ws: Optional[torch.Tensor] = None, kernel: int = 0) -> torch.Tensor:
    """lora_linear_pop with an epilogue op on the bf16 output y (eggroll_lora_linear_pop_epi_sel):
    "silu": silu(y); "gelu": gelu(y, approximate="tanh"); "gelu_erf": gelu(y) (exact, torch's bits); "mul": res * y; "res": res + y; "gated": res + gate[row // rows_per_group] * y.  With res given and
    out None the result is written into res (in place, as the residual adds it replaces).
    "res32" / "gated32": res is the fp32 residual stream, updated in place (res + y /
    fma(gate, y, res), gate fp32); out (optional) receives its bf16 shadow; returns res.
    kernel: 0 automatic, 8 / 10 the 256x256 / 256x320 8-phase kernels (A/B measurement)."""
    _dev(x, "lora_linear_pop_epi(x)", torch.bfloat16)
    _dev(W, "lora_linear_pop_epi(W)", torch.bfloat16)
    M, Kd = x.shape
    N = W.shape[0]
    code = EPI[epi]
    f32res = code in (4, 5)
    if res is not None:
        _dev(res, "lora_linear_pop_epi(res)", torch.float32 if f32res else torch.bfloat16)
        if res.shape[-1] != N or res.numel() != M * N:
            raise ValueError(f"res {tuple(res.shape)} does not match [{M}, {N}]")
    if f32res:
        if res is None or (code == 5 and (gate is None or gate.dtype != torch.float32)):
            raise ValueError(f"lora_linear_pop_epi({epi}): needs an fp32 res (and an fp32 gate)")
        if out is not None:
            _dev(out, "lora_linear_pop_epi(out)", torch.bfloat16)
    elif out is None:
        out = res if res is not None and code in (2, 3, 7) else torch.empty((M, N), dtype=torch.bfloat16, device=x.device)
    pg, gst = _row_ptr(gate, "lora_linear_pop_epi(gate)", N, allow_f32=code == 5) if gate is not None else (None, 0)
    if r > 0:
        _dev(theta_pop, "lora_linear_pop_epi(theta_pop)", torch.float32)
        need = lora_workspace_numel(M, Kd, r, rows_per_member)
        if T_ws is None or T_ws.numel() < need:
            T_ws = torch.empty(need, dtype=torch.float32, device=x.device)
    _lib.call("eggroll_lora_linear_pop_epi_sel", x.data_ptr(), x.stride(0), W.data_ptr(), W.stride(0), _p(bias),
              _p(theta_pop) if r > 0 else None, theta_pop.stride(0) if r > 0 else 0, offA, offB, r, float(scale),
              rows_per_member, M, N, Kd, _p(out), N, _p(T_ws) if r > 0 else None, code,
              _p(res), N if res is not None else 0, pg, gst or N, int(rows_per_group), int(kernel), _stream(x.device))
    return res if f32res else out


def lora_gemm_epi(x: torch.Tensor, W: torch.Tensor, bias: Optional[torch.Tensor], T: Optional[torch.Tensor],
                  theta_pop: Optional[torch.Tensor], offB: int, r: int, scale: float, rows_per_member: int, epi: str,
                  res: Optional[torch.Tensor] = None, gate: Optional[torch.Tensor] = None, rows_per_group: int = 1,
                  out: Optional[torch.Tensor] = None, kernel: int = 0) -> torch.Tensor:
    """lora_linear_pop_epi's GEMM with T = X A_k^T given (eggroll_lora_gemm_epi_sel): the same kernel and bits
    as the second of lora_linear_pop_epi's two launches.  Same res / out / return conventions."""
    _dev(x, "lora_gemm_epi(x)", torch.bfloat16)
    _dev(W, "lora_gemm_epi(W)", torch.bfloat16)
    M, Kd = x.shape
    N = W.shape[0]
    code = EPI[epi]
    if code == 0:
        raise ValueError("lora_gemm_epi: needs an epilogue op (use lora_gemm)")
    f32res = code in (4, 5)
    if res is not None:
        _dev(res, "lora_gemm_epi(res)", torch.float32 if f32res else torch.bfloat16)
        if res.shape[-1] != N or res.numel() != M * N:
            raise ValueError(f"res {tuple(res.shape)} does not match [{M}, {N}]")
    if f32res:
        if res is None or (code == 5 and (gate is None or gate.dtype != torch.float32)):
            raise ValueError(f"lora_gemm_epi({epi}): needs an fp32 res (and an fp32 gate)")
        if out is not None:
            _dev(out, "lora_gemm_epi(out)", torch.bfloat16)
    elif out is None:
        out = res if res is not None and code in (2, 3, 7) else torch.empty((M, N), dtype=torch.bfloat16, device=x.device)
    pg, gst = _row_ptr(gate, "lora_gemm_epi(gate)", N, allow_f32=code == 5) if gate is not None else (None, 0)
    if r > 0:
        _dev(theta_pop, "lora_gemm_epi(theta_pop)", torch.float32)
        _dev(T, "lora_gemm_epi(T)", torch.float32)
    _lib.call("eggroll_lora_gemm_epi_sel", x.data_ptr(), x.stride(0), W.data_ptr(), W.stride(0), _p(bias),
              _p(T) if r > 0 else None, _p(theta_pop) if r > 0 else None, theta_pop.stride(0) if r > 0 else 0, offB, r,
              float(scale), rows_per_member, M, N, Kd, _p(out), N, code, _p(res), N if res is not None else 0, pg,
              gst or N, int(rows_per_group), int(kernel), _stream(x.device))
    return res if f32res else out


def lora_workspace_numel(M: int, K: int, r: int, rows_per_member: int) -> int:
    """fp32 elements of the eggroll_lora_linear_pop workspace (T, or the fused path's A_k images)."""
    nbytes = int(_lib.load().eggroll_lora_workspace_bytes(M, K, r, rows_per_member))
    return max(1, -(-nbytes // 4))


def lora_fused(M: int, N: int, K: int, r: int, rows_per_member: int, kernel: int = 0) -> bool:
    """True when eggroll_lora_linear_pop_sel runs the projection inside the 8-phase GEMM (mirrors
    fused_ok in eggroll_lora.hip): only with kernel 12 — the automatic choice is the two-pass
    k_lora_project + k_lora_gemm8, which measured faster at every Sana shape."""
    return kernel == 12 and r in (1, 2) and rows_per_member >= 256 and K % 64 == 0


def lora_gemm(x: torch.Tensor, W: torch.Tensor, bias: Optional[torch.Tensor], T: Optional[torch.Tensor],
              theta_pop: Optional[torch.Tensor], offB: int, r: int, scale: float, rows_per_member: int,
              out: Optional[torch.Tensor] = None, kernel: int = 0) -> torch.Tensor:
    """The MFMA GEMM + fused LoRA epilogue alone, given T = X A_k^T (from lora_project)."""
    _dev(x, "lora_gemm(x)", torch.bfloat16)
    _dev(W, "lora_gemm(W)", torch.bfloat16)
    M, K = x.shape
    N = W.shape[0]
    if out is None:
        out = torch.empty((M, N), dtype=torch.bfloat16, device=x.device)
    ld_t = theta_pop.stride(0) if (r > 0 and theta_pop is not None) else 0
    _lib.call("eggroll_lora_gemm_sel", x.data_ptr(), x.stride(0), W.data_ptr(), W.stride(0), _p(bias),
              _p(T) if r > 0 else None, _p(theta_pop) if r > 0 else None, ld_t, offB, r, float(scale),
              rows_per_member, M, N, K, out.data_ptr(), out.stride(0), int(kernel), _stream(x.device))
    return out


def gemm_tile_for(M: int, N: int, r: int = 2, rows_per_member: int = 1 << 30, epi: Optional[str] = None) -> int:
    """Kernel libeggroll's automatic choice uses for an M x N LoRA GEMM (mirrors lora_gemm_impl / gemm_epi_impl
    / gemm8_auto): 8 = the 8-phase 256x256 kernel, 10 = the 8-phase 256x320 kernel, 128 = the 128x128
    one-barrier tile (no epilogue op only)."""
    if epi is None and (M // 256) * ((N + 255) // 256) < 512:
        return 128
    if not (r == 0 or (r <= 2 and rows_per_member >= 256)) or epi in ("res", "gated", "mul"):
        return 8
    tm = -(-M // 256)
    rounds8, rounds10 = -(-(tm * -(-N // 256)) // 256), -(-(tm * -(-N // 320)) // 256)
    return 10 if 122 * rounds10 < 100 * rounds8 else 8


def lora_project(x: torch.Tensor, theta_pop: torch.Tensor, offA: int, r: int, rows_per_member: int,
                 out: Optional[torch.Tensor] = None) -> torch.Tensor:
    _dev(x, "lora_project(x)", torch.bfloat16)
    _dev(theta_pop, "lora_project(theta_pop)", torch.float32)
    M, K = x.shape
    if out is None:
        out = torch.empty((M, r), dtype=torch.float32, device=x.device)
    _lib.call("eggroll_lora_project", x.data_ptr(), x.stride(0), theta_pop.data_ptr(), theta_pop.stride(0), offA, r,
              rows_per_member, M, K, out.data_ptr(), _stream(x.device))
    return out


def lora_project_multi(x: torch.Tensor, theta_pop: torch.Tensor, offAs: Sequence[int], r: int, rows_per_member: int,
                       out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """T_l = X A_{k,l}^T for several LoRA linears reading the same x, x read once (MFMA, A as bf16 hi + lo:
    equal to lora_project to fp32 rounding).  Returns [n_lin, M, r] fp32."""
    _dev(x, "lora_project_multi(x)", torch.bfloat16)
    _dev(theta_pop, "lora_project_multi(theta_pop)", torch.float32)
    M, Kd = x.shape
    n = len(offAs)
    if out is None:
        out = torch.empty((n, M, r), dtype=torch.float32, device=x.device)
    _dev(out, "lora_project_multi(out)", torch.float32)
    if out.numel() < n * M * r:
        raise ValueError("lora_project_multi: out too small")
    offs = np.asarray([int(o) for o in offAs], dtype=np.int64)
    _lib.call("eggroll_lora_project_multi", x.data_ptr(), x.stride(0), theta_pop.data_ptr(), theta_pop.stride(0),
              offs.ctypes.data, n, r, rows_per_member, M, Kd, out.data_ptr(), _stream(x.device))
    return out


def lora_expand(T: torch.Tensor, theta_pop: torch.Tensor, offB: int, r: int, scale: float, rows_per_member: int,
                y: torch.Tensor) -> torch.Tensor:
    _dev(T, "lora_expand(T)", torch.float32)
    _dev(y, "lora_expand(y)", torch.bfloat16)
    M, N = y.shape
    _lib.call("eggroll_lora_expand", T.data_ptr(), theta_pop.data_ptr(), theta_pop.stride(0), offB, r, float(scale),
              rows_per_member, M, N, y.data_ptr(), y.stride(0), _stream(y.device))
    return y


def lora_delta_f32(x: torch.Tensor, A: torch.Tensor, lda_member: int, B: torch.Tensor, ldb_member: int, r: int,
                   scale: float, rows_per_member: int, y: torch.Tensor) -> torch.Tensor:
    """y += scale * (x A_k^T) B_k^T in fp32 (eggroll_lora_delta_f32), k = row // rows_per_member; A / B point
    at member 0's lora_A [r][K] / lora_B [N][r] (a theta_pop column slice or the module's own weights) with
    member strides lda_member / ldb_member (0: one adapter for all rows).  x [M, K], y [M, N] fp32, rows with
    unit column stride; y is updated in place and returned."""
    _dev(x, "lora_delta_f32(x)", torch.float32, contiguous=False)
    _dev(y, "lora_delta_f32(y)", torch.float32, contiguous=False)
    _dev(A, "lora_delta_f32(A)", torch.float32, contiguous=False)
    _dev(B, "lora_delta_f32(B)", torch.float32, contiguous=False)
    M, Kd = x.shape
    if y.shape[0] != M or x.stride(1) != 1 or y.stride(1) != 1:
        raise ValueError(f"lora_delta_f32: x {tuple(x.shape)} / y {tuple(y.shape)} must have M rows of unit stride")
    N = y.shape[1]
    if M:
        n_members = (M - 1) // rows_per_member + 1
        for t, name, ld, need in ((A, "A", lda_member, r * Kd), (B, "B", ldb_member, N * r)):
            # the last member's adapter must lie inside the tensor the pointer came from
            if (n_members - 1) * ld + need > t.untyped_storage().nbytes() // 4 - t.storage_offset():
                raise ValueError(f"lora_delta_f32: {name} too small for {n_members} members")
    _lib.call("eggroll_lora_delta_f32", x.data_ptr(), x.stride(0), A.data_ptr(), lda_member, B.data_ptr(), ldb_member,
              r, float(scale), rows_per_member, M, N, Kd, y.data_ptr(), y.stride(0), _stream(y.device))
    return y


class OpTimer:
    """Opt-in live timing of the model-side libeggroll kernels (bench.py's per-kernel HBM table):
    HIP events on the launching stream around each call + its ALGORITHMIC bytes (every input read
    once, every output written once)."""

    active = False
    records: List[tuple] = []

    @classmethod
    def reset(cls, active: bool):
        cls.active, cls.records = active, []

    @classmethod
    def begin(cls):
        if not cls.active:
            return None
        e = torch.cuda.Event(enable_timing=True)
        e.record()
        return e

    @classmethod
    def end(cls, e0, name: str, nbytes: float, shape: str = "", flops: float = 0.0):
        if e0 is None:
            return
        e1 = torch.cuda.Event(enable_timing=True)
        e1.record()
        cls.records.append((name, e0, e1, float(nbytes), shape, float(flops)))

    @classmethod
    def summary(cls, peak_gbps: float = 8000.0) -> Dict[str, Dict[str, float]]:
        torch.cuda.synchronize()
        out: Dict[str, Dict[str, float]] = {}
        for name, e0, e1, nb, shape, fl in cls.records:
            ms = e0.elapsed_time(e1)
            for d in (out.setdefault(name, {"launches": 0, "total_ms": 0.0, "bytes": 0.0, "flops": 0.0, "shapes": {}}),):
                d["launches"] += 1
                d["total_ms"] += ms
                d["bytes"] += nb
                d["flops"] += fl
                sd = d["shapes"].setdefault(shape, {"launches": 0, "total_ms": 0.0, "bytes": 0.0, "flops": 0.0})
                sd["launches"] += 1
                sd["total_ms"] += ms
                sd["bytes"] += nb
                sd["flops"] += fl
        for d in out.values():
            for x in [d] + list(d["shapes"].values()):
                x["avg_us"] = 1e3 * x["total_ms"] / x["launches"]
                x["GBps"] = x["bytes"] / (x["total_ms"] * 1e6) if x["total_ms"] > 0 else float("nan")
                x["frac"] = x["GBps"] / peak_gbps
                if x["flops"] > 0:  # MFMA-bound ops: useful FLOP rate against the dense bf16 peak
                    x["tflops"] = x["flops"] / (x["total_ms"] * 1e9)
                    x["mfma_frac"] = x["tflops"] / 2500.0
                else:
                    x.pop("flops")
            top = sorted(d["shapes"].items(), key=lambda kv: -kv[1]["total_ms"])[:4]
            d["shapes"] = {k: {kk: round(vv, 3) for kk, vv in v.items()} for k, v in top}
        return out


# ---------------------------------------------------------------------------------------
# model-side fused op: channels-last depthwise conv (+SiLU on load, +GLU gate)
# ---------------------------------------------------------------------------------------


def dwconv_nhwc(x: torch.Tensor, w_t: torch.Tensor, bias: Optional[torch.Tensor], ks: int, pre_silu: bool,
                glu: bool, out: Optional[torch.Tensor] = None, kernel: int = 0, ldo: int = 0) -> torch.Tensor:
    """x [B,H,W,C] bf16 contiguous; w_t [ks*ks, C] bf16; returns [B,H,W,C or C/2].
    kernel: block order, 0 auto, 1 channel-fastest, 2 column sweep (eggroll_dwconv_nhwc_sel).
    ldo > 0: output channel stride (eggroll_dwconv_nhwc_ex): returns [B,H,W,ldo] whose channels past
    C (C/2) are zeros."""
    _dev(x, "dwconv(x)", torch.bfloat16)
    _dev(w_t, "dwconv(w_t)", torch.bfloat16)
    B, H, W, C = x.shape
    if w_t.shape != (ks * ks, C):
        raise ValueError(f"w_t {tuple(w_t.shape)} != ({ks * ks}, {C})")
    if bias is not None:
        _dev(bias, "dwconv(bias)", torch.bfloat16)
    co = C // 2 if glu else C
    ldo = ldo or co
    if out is None:
        out = torch.empty((B, H, W, ldo), dtype=torch.bfloat16, device=x.device)
    elif out.shape != (B, H, W, ldo) or not out.is_contiguous():
        raise ValueError(f"dwconv(out) {tuple(out.shape)} != ({B}, {H}, {W}, {ldo}) contiguous")
    e0 = OpTimer.begin()
    _lib.call("eggroll_dwconv_nhwc_ex", x.data_ptr(), w_t.data_ptr(), _p(bias), B, H, W, C, ks, int(pre_silu),
              int(glu), out.data_ptr(), ldo, int(kernel), _stream(x.device))
    OpTimer.end(e0, f"dwconv_nhwc<{ks},{int(pre_silu)},{int(glu)}>", 2.0 * B * H * W * (C + co), f"{B}x{H}x{W}x{C}")
    return out


def dwconv_pw_nhwc(x: torch.Tensor, w_t: torch.Tensor, pw: torch.Tensor, ks: int,
                   out: Optional[torch.Tensor] = None, kernel: int = 0) -> torch.Tensor:
    """Depthwise ks x ks conv (no bias) then grouped 1x1 conv (groups of 32): x [B,H,W,C] bf16,
    w_t [ks*ks, C], pw [C/32, 32, 32] ([group][out][in]) -> [B,H,W,C] (eggroll_dwconv_pw_nhwc)."""
    _dev(x, "dwconv_pw(x)", torch.bfloat16)
    _dev(w_t, "dwconv_pw(w_t)", torch.bfloat16)
    _dev(pw, "dwconv_pw(pw)", torch.bfloat16)
    x, pw = x.contiguous(), pw.contiguous()
    B, H, W, C = x.shape
    if w_t.shape != (ks * ks, C) or pw.shape != (C // 32, 32, 32) or C % 32:
        raise ValueError(f"dwconv_pw: w_t {tuple(w_t.shape)} / pw {tuple(pw.shape)} do not match C={C}, ks={ks}")
    if out is None:
        out = torch.empty_like(x)
    e0 = OpTimer.begin()
    _lib.call("eggroll_dwconv_pw_nhwc_sel", x.data_ptr(), w_t.data_ptr(), pw.data_ptr(), B, H, W, C, ks,
              out.data_ptr(), int(kernel), _stream(x.device))
    OpTimer.end(e0, f"dwconv_pw_nhwc<{ks}>", 4.0 * B * H * W * C, f"{B}x{H}x{W}x{C}")
    return out


def _row_ptr(t: Optional[torch.Tensor], what: str, C: int, allow_f32: bool = False):
    """Pointer + row stride of a [groups, C]-shaped (possibly strided) bf16 (or, allow_f32, fp32) view."""
    if t is None:
        return None, 0
    ok = (torch.bfloat16, torch.float32) if allow_f32 else (torch.bfloat16,)
    if t.device.type != "cuda" or t.dtype not in ok or t.stride(-1) != 1:
        raise _lib.EggrollError(f"{what}: expected a {'bf16 / fp32' if allow_f32 else 'bf16'} device view with "
                                f"unit inner stride")
    stride = t.stride(0) if t.dim() > 1 and t.shape[0] > 1 else C
    return t.data_ptr(), stride


ACT = {None: 0, "none": 0, "relu": 1, "silu": 2}


def rownorm(x: torch.Tensor, eps: float, layer: bool = False, w: Optional[torch.Tensor] = None,
            b: Optional[torch.Tensor] = None, mscale: Optional[torch.Tensor] = None,
            mshift: Optional[torch.Tensor] = None, rows_per_group: int = 1, act=None,
            res: Optional[torch.Tensor] = None, out: Optional[torch.Tensor] = None,
            shadow: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Fused (RMS|Layer)Norm over the last dim [+w][*(1+mscale[g])][+mshift[g]][+b][act][+res].
    mscale / mshift: [groups, C] views (rows `mstride` apart), g = row // rows_per_group.
    x may be fp32 (the Sana fp32 residual stream) and mscale / mshift fp32 (the fp32 modulation); the
    output is bf16 — unless res is fp32 (the DC-AE fp32 residual stream): then the output is fp32
    (default: written into res in place) and `shadow` (optional bf16) receives its bf16 copy
    (eggroll_rownorm_ex)."""
    if x.dtype not in (torch.bfloat16, torch.float32):
        raise _lib.EggrollError("rownorm(x): expected bf16 or fp32")
    _dev(x, "rownorm(x)", x.dtype)
    C = x.shape[-1]
    rows = x.numel() // C
    of32 = res is not None and res.dtype == torch.float32
    if out is None:
        out = res if of32 else torch.empty(x.shape, dtype=torch.bfloat16, device=x.device)
    _dev(out, "rownorm(out)", torch.float32 if of32 else torch.bfloat16)
    if shadow is not None:
        if not of32:
            raise ValueError("rownorm: shadow needs an fp32 res / output")
        _dev(shadow, "rownorm(shadow)", torch.bfloat16)
    for t, nm in ((w, "w"), (b, "b")):
        if t is not None:
            _dev(t, f"rownorm({nm})", torch.bfloat16)
    if res is not None:
        _dev(res, "rownorm(res)", res.dtype)
    ps, st1 = _row_ptr(mscale, "rownorm(mscale)", C, allow_f32=True)
    ph, st2 = _row_ptr(mshift, "rownorm(mshift)", C, allow_f32=True)
    if ps is not None and ph is not None and (st1 != st2 or mscale.dtype != mshift.dtype):
        raise ValueError("mscale / mshift must share a row stride and a dtype")
    mf32 = int(any(t is not None and t.dtype == torch.float32 for t in (mscale, mshift)))
    xf32 = int(x.dtype == torch.float32)
    e0 = OpTimer.begin()
    _lib.call("eggroll_rownorm_ex", x.data_ptr(), xf32, rows, C, float(eps), int(bool(layer)), _p(w), _p(b), ps, ph,
              st1 or st2 or C, mf32, int(rows_per_group), ACT[act], _p(res), int(of32), out.data_ptr(), int(of32),
              _p(shadow), _stream(x.device))
    OpTimer.end(e0, f"rownorm(C={C})", (2.0 + 2 * xf32) * rows * C + rows * C * (
        (8.0 + (2 if shadow is not None else 0)) if of32 else (4.0 if res is not None else 2.0)), f"rows{rows}")
    return out


def qk_norm_rope_(x: torch.Tensor, w: torch.Tensor, eps: float, cos: torch.Tensor, sin: torch.Tensor,
                  heads: int) -> torch.Tensor:
    """In place on x [rows, >= heads*128] bf16 (row stride x.stride(0)): per-head RMS norm * w [128], then
    the rotation of adjacent pairs by cos / sin [tab_rows, 64] fp32 (table row = row % tab_rows) —
    eggroll_qk_norm_rope (the Z-Image q / k path)."""
    _dev(x, "qk_norm_rope(x)", torch.bfloat16, contiguous=False)
    _dev(w, "qk_norm_rope(w)", torch.bfloat16)
    _dev(cos, "qk_norm_rope(cos)", torch.float32)
    _dev(sin, "qk_norm_rope(sin)", torch.float32)
    if x.dim() != 2 or x.stride(1) != 1 or cos.shape != sin.shape or cos.shape[-1] != 64 or w.numel() != 128:
        raise ValueError(f"qk_norm_rope: x {tuple(x.shape)}, w {tuple(w.shape)}, tables {tuple(cos.shape)}")
    e0 = OpTimer.begin()
    _lib.call("eggroll_qk_norm_rope", x.data_ptr(), x.stride(0), x.shape[0], int(heads), 128, float(eps), w.data_ptr(),
              cos.data_ptr(), sin.data_ptr(), cos.numel() // 64, _stream(x.device))
    OpTimer.end(e0, "qk_norm_rope", 4.0 * x.shape[0] * heads * 128, f"rows{x.shape[0]}")
    return x


def qk_norm_rope_kv(x: torch.Tensor, w: torch.Tensor, eps: float, cos: torch.Tensor, sin: torch.Tensor, heads: int,
                    hscale: Optional[torch.Tensor] = None, out: Optional[torch.Tensor] = None, rows_per_seq: int = 1,
                    row0: int = 0, vin: Optional[torch.Tensor] = None, vout: Optional[torch.Tensor] = None) -> None:
    """eggroll_qk_norm_rope_kv: x [rows, >= heads*128] bf16 (row stride x.stride(0)); hscale fp32 [heads]
    (optional output multiplier); out (optional) a [seq, ltot, C] bf16 cache: row r goes to
    out[r // rows_per_seq, row0 + r % rows_per_seq]; vin (optional, [rows, ...] like x) copied into vout
    (same geometry as out) at the same positions."""
    _dev(x, "qk_norm_rope_kv(x)", torch.bfloat16, contiguous=False)
    _dev(w, "qk_norm_rope_kv(w)", torch.bfloat16)
    if x.dim() != 2 or x.stride(1) != 1 or cos.shape != sin.shape or cos.shape[-1] != 64 or w.numel() != 128:
        raise ValueError(f"qk_norm_rope_kv: x {tuple(x.shape)}, w {tuple(w.shape)}, tables {tuple(cos.shape)}")
    if hscale is not None:
        _dev(hscale, "qk_norm_rope_kv(hscale)", torch.float32)
    ob = ol = 0
    if out is not None:
        _dev(out, "qk_norm_rope_kv(out)", torch.bfloat16)
        if out.dim() != 3 or out.shape[0] * rows_per_seq != x.shape[0] or row0 + rows_per_seq > out.shape[1]:
            raise ValueError(f"qk_norm_rope_kv: out {tuple(out.shape)} vs {x.shape[0]} rows of {rows_per_seq}")
        ob, ol = out.stride(0), out.stride(1)
    if vin is not None:
        _dev(vin, "qk_norm_rope_kv(vin)", torch.bfloat16, contiguous=False)
        if vout is None or vout.shape != out.shape or vout.stride() != out.stride() or vin.shape[0] != x.shape[0]:
            raise ValueError("qk_norm_rope_kv: vin needs a vout shaped like out")
    e0 = OpTimer.begin()
    _lib.call("eggroll_qk_norm_rope_kv", x.data_ptr(), x.stride(0), x.shape[0], int(heads), 128, float(eps), w.data_ptr(),
              cos.data_ptr(), sin.data_ptr(), cos.numel() // 64, _p(hscale), _p(out), ob, ol, int(rows_per_seq),
              int(row0), _p(vin), vin.stride(0) if vin is not None else 0, _p(vout), _stream(x.device))
    OpTimer.end(e0, "qk_norm_rope", (4.0 + (4.0 if vin is not None else 0.0)) * x.shape[0] * heads * 128,
                f"rows{x.shape[0]}")


def gated_residual_(x: torch.Tensor, y: torch.Tensor, gate: torch.Tensor, rows_per_group: int) -> torch.Tensor:
    """x += gate[g] * y in place (g = row // rows_per_group); gate a [groups, C] view."""
    _dev(x, "gated_residual(x)", torch.bfloat16)
    _dev(y, "gated_residual(y)", torch.bfloat16)
    C = x.shape[-1]
    pg, st = _row_ptr(gate, "gated_residual(gate)", C)
    e0 = OpTimer.begin()
    _lib.call("eggroll_gated_residual", x.data_ptr(), y.data_ptr(), pg, st, x.numel() // C, C, int(rows_per_group),
              _stream(x.device))
    OpTimer.end(e0, "gated_residual", 6.0 * x.numel())
    return x



def gated_residual_f32_(x: torch.Tensor, y: torch.Tensor, gate: Optional[torch.Tensor], rows_per_group: int = 1,
                        shadow: Optional[torch.Tensor] = None) -> torch.Tensor:
    """fp32 residual stream update in place: x = fma(gate[g], y, x) (gate bf16 / fp32 [groups, C] view;
    None: x += y), y bf16; shadow (optional bf16, x's shape) receives bf16(x)
    (eggroll_gated_residual_f32 — the unfused form of the EPI_RES32 / EPI_GATED32 GEMM epilogues)."""
    _dev(x, "gated_residual_f32(x)", torch.float32)
    _dev(y, "gated_residual_f32(y)", torch.bfloat16)
    C = x.shape[-1]
    if y.numel() != x.numel() or y.shape[-1] != C:
        raise ValueError(f"gated_residual_f32: y {tuple(y.shape)} does not match x {tuple(x.shape)}")
    if shadow is not None:
        _dev(shadow, "gated_residual_f32(shadow)", torch.bfloat16)
    pg, st = _row_ptr(gate, "gated_residual_f32(gate)", C, allow_f32=True)
    e0 = OpTimer.begin()
    _lib.call("eggroll_gated_residual_f32", x.data_ptr(), y.data_ptr(), pg,
              int(gate is not None and gate.dtype == torch.float32), st or C, x.numel() // C, C, int(rows_per_group),
              _p(shadow), _stream(x.device))
    OpTimer.end(e0, "gated_residual_f32", (10.0 + (2 if shadow is not None else 0)) * x.numel(), f"rows{x.numel() // C}")
    return x

def resid_layernorm_(h: torch.Tensor, y: Optional[torch.Tensor], w: torch.Tensor, b: torch.Tensor, eps: float,
                     out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """h [..., C] fp32 (rows may be strided: a [n, T, C] stream or its [:, 0] rows) += y (bf16, same row
    count, or None) in place; returns bf16 layer_norm(h) * w + b [rows, C] (eggroll_resid_layernorm)."""
    _dev(h, "resid_layernorm(h)", torch.float32, contiguous=False)   # rows may be strided (row stride passed)
    C = h.shape[-1]
    h2 = h if h.dim() == 2 else h.view(-1, C)   # a view: the in-place add must land in h
    if h2.stride(1) != 1:
        raise ValueError(f"resid_layernorm: h must be rows of C unit-stride channels, got {tuple(h.shape)} {h.stride()}")
    rows = h2.shape[0]
    ldy = 0
    if y is not None:
        _dev(y, "resid_layernorm(y)", torch.bfloat16)
        y2 = y.reshape(-1, C)
        if y2.shape[0] != rows or y2.stride(1) != 1:
            raise ValueError(f"resid_layernorm: y {tuple(y.shape)} does not match h rows {rows}")
        ldy = y2.stride(0)
    _dev(w, "resid_layernorm(w)", torch.bfloat16)
    _dev(b, "resid_layernorm(b)", torch.bfloat16)
    if w.numel() != C or b.numel() != C:
        raise ValueError("resid_layernorm: w / b must have C entries")
    if out is None:
        out = torch.empty((rows, C), dtype=torch.bfloat16, device=h.device)
    e0 = OpTimer.begin()
    _lib.call("eggroll_resid_layernorm", h2.data_ptr(), h2.stride(0), _p(y2 if y is not None else None), ldy, rows, C,
              float(eps), w.data_ptr(), b.data_ptr(), out.data_ptr(), _stream(h.device))
    OpTimer.end(e0, "resid_layernorm", float(rows) * C * ((8 if y is not None else 4) + 2 + 2))
    return out


def upshortcut_add_(y: torch.Tensor, x: torch.Tensor) -> torch.Tensor:
    """y [B,2H,2W,Cout] += pixel_shuffle(repeat_interleave(x [B,H,W,Cin])) in place (NHWC)."""
    _dev(y, "upshortcut(y)", torch.bfloat16)
    _dev(x, "upshortcut(x)", torch.bfloat16)
    B, H, W, Cin = x.shape
    Cout = y.shape[-1]
    if y.shape[:3] != (B, 2 * H, 2 * W):
        raise ValueError(f"upshortcut: y {tuple(y.shape)} vs x {tuple(x.shape)}")
    e0 = OpTimer.begin()
    _lib.call("eggroll_upshortcut_add", y.data_ptr(), x.data_ptr(), B, H, W, Cin, Cout, _stream(x.device))
    OpTimer.end(e0, "upshortcut_add", 4.0 * y.numel() + 2.0 * x.numel())
    return y


def subpixel_shortcut(y4: torch.Tensor, x: torch.Tensor, out: Optional[torch.Tensor] = None,
                      bias: Optional[torch.Tensor] = None) -> torch.Tensor:
    """y4 [B,H+1,W+1,4*Cout] (bias-free phase conv output), x [B,H,W,Cin], bias [Cout] or None
    -> out [B,2H,2W,Cout] (NHWC)."""
    _dev(y4, "subpixel(y4)", torch.bfloat16)
    _dev(x, "subpixel(x)", torch.bfloat16)
    B, H, W, Cin = x.shape
    if y4.shape[:3] != (B, H + 1, W + 1) or y4.shape[3] % 4:
        raise ValueError(f"subpixel: y4 {tuple(y4.shape)} vs x {tuple(x.shape)}")
    Cout = y4.shape[3] // 4
    if bias is not None:
        _dev(bias, "subpixel(bias)", torch.bfloat16)
        if bias.numel() != Cout:
            raise ValueError(f"subpixel: bias has {bias.numel()} entries, Cout = {Cout}")
    if out is None:
        out = torch.empty((B, 2 * H, 2 * W, Cout), dtype=torch.bfloat16, device=x.device)
    e0 = OpTimer.begin()
    _lib.call("eggroll_subpixel_shortcut", y4.data_ptr(), x.data_ptr(), _p(bias), out.data_ptr(), B, H, W, Cin,
              Cout, _stream(x.device))
    OpTimer.end(e0, "subpixel_shortcut", 2.0 * (y4.numel() + x.numel() + out.numel()), f"{tuple(x.shape)}->{Cout}")
    return out


def subpixel_shortcut_f32(y4: torch.Tensor, x32: torch.Tensor, bias: Optional[torch.Tensor] = None,
                          shadow: Optional[torch.Tensor] = None) -> torch.Tensor:
    """subpixel_shortcut on the DC-AE fp32 residual stream: x32 [B,H,W,Cin] fp32 (shortcut source) ->
    out [B,2H,2W,Cout] fp32; shadow (optional [B,2H,2W,Cout] bf16) receives bf16(out)."""
    _dev(y4, "subpixel_f32(y4)", torch.bfloat16)
    _dev(x32, "subpixel_f32(x)", torch.float32)
    B, H, W, Cin = x32.shape
    if y4.shape[:3] != (B, H + 1, W + 1) or y4.shape[3] % 4:
        raise ValueError(f"subpixel_f32: y4 {tuple(y4.shape)} vs x {tuple(x32.shape)}")
    Cout = y4.shape[3] // 4
    if bias is not None:
        _dev(bias, "subpixel_f32(bias)", torch.bfloat16)
    out = torch.empty((B, 2 * H, 2 * W, Cout), dtype=torch.float32, device=x32.device)
    if shadow is not None:
        _dev(shadow, "subpixel_f32(shadow)", torch.bfloat16)
        if shadow.shape != out.shape:
            raise ValueError("subpixel_f32: shadow shape")
    e0 = OpTimer.begin()
    _lib.call("eggroll_subpixel_shortcut_f32", y4.data_ptr(), x32.data_ptr(), _p(bias), out.data_ptr(), _p(shadow), B,
              H, W, Cin, Cout, _stream(x32.device))
    OpTimer.end(e0, "subpixel_shortcut_f32", 2.0 * y4.numel() + 4.0 * x32.numel() + (6.0 if shadow is not None else 4.0)
                * out.numel(), f"{tuple(x32.shape)}->{Cout}")
    return out


_LA_WS: Dict[str, torch.Tensor] = {}


def linear_attention(q: torch.Tensor, k: torch.Tensor, v: torch.Tensor, B: int, N: int, heads: int,
                     hstride: int, relu_qk: bool, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """ReLU linear attention (head dim 32) over strided bf16 views q/k/v [B*N, ...] whose head h
    starts at column h*hstride.  Returns [B*N, heads*32] bf16."""
    for t, nm in ((q, "q"), (k, "k"), (v, "v")):
        if t.device.type != "cuda" or t.dtype != torch.bfloat16 or t.stride(-1) != 1:
            raise _lib.EggrollError(f"linear_attention({nm}): expected a bf16 device view with unit inner stride")
    ld = q.stride(0)
    if k.stride(0) != ld or v.stride(0) != ld:
        raise ValueError("linear_attention: q/k/v must share a row stride")
    if out is None:
        out = torch.empty((B * N, heads * 32), dtype=torch.bfloat16, device=q.device)
    nbytes = int(_lib.load().eggroll_linear_attention_workspace_bytes(B, N, heads))
    key = str(q.device)
    ws = _LA_WS.get(key)
    if ws is None or ws.numel() < nbytes:
        ws = _LA_WS[key] = torch.empty(max(nbytes, 16), dtype=torch.uint8, device=q.device)
    e0 = OpTimer.begin()
    _lib.call("eggroll_linear_attention", q.data_ptr(), k.data_ptr(), v.data_ptr(), ld, hstride, B, N, heads,
              int(bool(relu_qk)), out.data_ptr(), out.stride(0), ws.data_ptr(), _stream(q.device))
    OpTimer.end(e0, "linear_attention", 2.0 * B * N * heads * 32 * 4, f"B{B} N{N} h{heads}")
    return out


def dcae_head(x: torch.Tensor, eps: float, norm_w: torch.Tensor, norm_b: torch.Tensor, conv_w: torch.Tensor,
              conv_b: Optional[torch.Tensor]) -> torch.Tensor:
    """Fused RMSNorm(+w,+b) -> ReLU -> 3x3 conv (C=128 -> 3, pad 1, +bias): x [B,H,W,128] NHWC bf16,
    conv_w [3,128,3,3] -> y [B,H,W,3] bf16 (NHWC)."""
    _dev(x, "dcae_head(x)", torch.bfloat16)
    for t, nm in ((norm_w, "norm_w"), (norm_b, "norm_b")):
        _dev(t, f"dcae_head({nm})", torch.bfloat16)
    if conv_b is not None:
        _dev(conv_b, "dcae_head(conv_b)", torch.bfloat16)
    x = x.contiguous()
    B, H, W, C = x.shape
    if tuple(conv_w.shape) != (3, C, 3, 3):
        raise ValueError(f"dcae_head: conv_w {tuple(conv_w.shape)} != (3, {C}, 3, 3)")
    wt = conv_w.permute(0, 2, 3, 1).contiguous()  # [o][ky][kx][c] (a view for channels-last weights)
    _dev(wt, "dcae_head(conv_w)", torch.bfloat16)
    y = torch.empty((B, H, W, 3), dtype=torch.bfloat16, device=x.device)
    e0 = OpTimer.begin()
    _lib.call("eggroll_dcae_head", x.data_ptr(), B, H, W, C, float(eps), norm_w.data_ptr(), norm_b.data_ptr(),
              wt.data_ptr(), _p(conv_b), y.data_ptr(), _stream(x.device))
    OpTimer.end(e0, "dcae_head", 2.0 * x.numel() + 2.0 * y.numel(), f"{tuple(x.shape)}")
    return y


def pack_conv3x3_weight(w: torch.Tensor, px: int) -> torch.Tensor:
    """[Cout, Cin, ks, ks] conv weight -> the implicit-GEMM operand [px*Cout, ks*(px+ks-1)*Cin] bf16 of
    eggroll_conv_nhwc: row p*Cout + o, column (ky*(px+ks-1) + tx)*Cin + c holds w[o, c, ky, tx - p]
    (zero where tx - p is outside 0..ks-1).  px = 1 is the channels-last weight itself."""
    Cout, Cin, ks = w.shape[0], w.shape[1], w.shape[-1]
    wt = w.permute(0, 2, 3, 1).to(torch.bfloat16)  # [o][ky][kx][c]
    tw = px + ks - 1
    out = torch.zeros((px, Cout, ks, tw, Cin), dtype=torch.bfloat16, device=w.device)
    for p in range(px):
        out[p, :, :, p:p + ks, :] = wt
    return out.reshape(px * Cout, ks * tw * Cin).contiguous()


def conv_nhwc(x: torch.Tensor, w_packed: torch.Tensor, bias: Optional[torch.Tensor], ks: int, px: int = 1,
              act: Optional[str] = None, out: Optional[torch.Tensor] = None, kernel: int = 0) -> torch.Tensor:
    """ks x ks conv (ks 2 or 3), zero pad 1, of x [B,H,W,Cin] NHWC bf16 -> [B, H+3-ks, W+3-ks, N/px].
    kernel: 0 auto, 1 tap-staged implicit GEMM, 2 halo-staged (eggroll_conv_nhwc_sel)."""
    _dev(x, "conv(x)", torch.bfloat16)
    _dev(w_packed, "conv(w)", torch.bfloat16)
    x = x.contiguous()
    B, H, W, Cin = x.shape
    N = w_packed.shape[0]
    if w_packed.shape[1] != ks * (px + ks - 1) * Cin or N % px:
        raise ValueError(f"conv: packed weight {tuple(w_packed.shape)} does not match Cin={Cin}, ks={ks}, px={px}")
    if bias is not None:
        _dev(bias, "conv(bias)", torch.bfloat16)
        if bias.numel() != N:
            raise ValueError(f"conv: bias has {bias.numel()} entries, need {N}")
    Ho, Wo, Cout = H + 3 - ks, W + 3 - ks, N // px
    if out is None:
        out = torch.empty((B, Ho, Wo, Cout), dtype=torch.bfloat16, device=x.device)
    e0 = OpTimer.begin()
    _lib.call("eggroll_conv_nhwc_sel", x.data_ptr(), w_packed.data_ptr(), _p(bias), B, H, W, Cin, N, ks, px,
              ACT[act], out.data_ptr(), int(kernel), _stream(x.device))
    OpTimer.end(e0, f"conv{ks}x{ks}", 2.0 * (x.numel() + out.numel()), f"{tuple(x.shape)}->{Cout} px{px}",
                flops=2.0 * B * Ho * Wo * Cout * ks * ks * Cin)
    return out


def conv2x2_subpixel(x: torch.Tensor, w4_packed: torch.Tensor, src: torch.Tensor, bias: Optional[torch.Tensor] = None,
                     shadow: Optional[torch.Tensor] = None, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """DC-AE up-block in one launch (eggroll_conv2x2_subpixel_nhwc): the bias-free ks-2 phase conv of x
    [B,H,W,Cin] bf16 (w4_packed [4*Cout][2][2][Cin]) with the sub-pixel interleave, bias and pixel-shuffle
    shortcut from src in its epilogue -> [B,2H,2W,Cout].  src bf16 (= x): bf16 out; src fp32 (the DC-AE
    fp32 residual stream): fp32 out and, when given, its bf16 shadow.  Bitwise equal to conv_nhwc(ks 2)
    followed by subpixel_shortcut / subpixel_shortcut_f32."""
    _dev(x, "conv2x2_subpixel(x)", torch.bfloat16)
    _dev(w4_packed, "conv2x2_subpixel(w)", torch.bfloat16)
    f32 = src.dtype == torch.float32
    _dev(src, "conv2x2_subpixel(src)", torch.float32 if f32 else torch.bfloat16)
    x = x.contiguous()
    B, H, W, Cin = x.shape
    N = w4_packed.shape[0]
    if w4_packed.shape[1] != 4 * Cin or N % 4 or tuple(src.shape) != (B, H, W, Cin):
        raise ValueError(f"conv2x2_subpixel: weight {tuple(w4_packed.shape)} / src {tuple(src.shape)} vs x {tuple(x.shape)}")
    Cout = N // 4
    if bias is not None:
        _dev(bias, "conv2x2_subpixel(bias)", torch.bfloat16)
        if bias.numel() != Cout:
            raise ValueError(f"conv2x2_subpixel: bias has {bias.numel()} entries, Cout = {Cout}")
    if shadow is not None:
        if not f32:
            raise ValueError("conv2x2_subpixel: shadow needs an fp32 src")
        _dev(shadow, "conv2x2_subpixel(shadow)", torch.bfloat16)
    if out is None:
        out = torch.empty((B, 2 * H, 2 * W, Cout), dtype=src.dtype, device=x.device)
    _dev(out, "conv2x2_subpixel(out)", src.dtype)
    e0 = OpTimer.begin()
    _lib.call("eggroll_conv2x2_subpixel_nhwc", x.data_ptr(), w4_packed.data_ptr(), _p(bias), src.data_ptr(), int(f32),
              B, H, W, Cin, Cout, out.data_ptr(), _p(shadow), _stream(x.device))
    OpTimer.end(e0, "conv2x2", 2.0 * x.numel() + out.element_size() * out.numel() + src.element_size() * src.numel(),
                f"{tuple(x.shape)}->{N} px1 +subpixel", flops=2.0 * B * (H + 1) * (W + 1) * N * 4 * Cin)
    return out


def conv3x3_nhwc(x: torch.Tensor, w_packed: torch.Tensor, bias: Optional[torch.Tensor], px: int,
                 act: Optional[str] = None, out: Optional[torch.Tensor] = None, kernel: int = 0) -> torch.Tensor:
    """3x3 conv (stride 1, pad 1) of x [B,H,W,Cin] NHWC bf16 with a pack_conv3x3_weight operand;
    bias [px*Cout] (the conv bias repeated px times) or None; act None / 'silu'.  -> [B,H,W,Cout]."""
    _dev(x, "conv3x3(x)", torch.bfloat16)
    _dev(w_packed, "conv3x3(w)", torch.bfloat16)
    x = x.contiguous()
    B, H, W, Cin = x.shape
    N = w_packed.shape[0]
    if w_packed.shape[1] != 3 * (px + 2) * Cin or N % px:
        raise ValueError(f"conv3x3: packed weight {tuple(w_packed.shape)} does not match Cin={Cin}, px={px}")
    if bias is not None:
        _dev(bias, "conv3x3(bias)", torch.bfloat16)
        if bias.numel() != N:
            raise ValueError(f"conv3x3: bias has {bias.numel()} entries, need {N}")
    Cout = N // px
    if out is None:
        out = torch.empty((B, H, W, Cout), dtype=torch.bfloat16, device=x.device)
    e0 = OpTimer.begin()
    _lib.call("eggroll_conv_nhwc_sel", x.data_ptr(), w_packed.data_ptr(), _p(bias), B, H, W, Cin, N, 3, px,
              ACT[act], out.data_ptr(), int(kernel), _stream(x.device))
    OpTimer.end(e0, "conv3x3", 2.0 * (x.numel() + out.numel()), f"{tuple(x.shape)}->{Cout} px{px}",
                flops=2.0 * B * H * W * Cout * 9 * Cin)
    return out


def conv3x3_rmsnorm_nhwc(x: torch.Tensor, w_packed: torch.Tensor, bias: Optional[torch.Tensor], px: int, eps: float,
                         norm_w: torch.Tensor, norm_b: Optional[torch.Tensor], res: torch.Tensor,
                         kernel: int = 0) -> torch.Tensor:
    """conv3x3_nhwc followed by RMSNorm over channels (* norm_w + norm_b) + res, in one launch
    (the DC-AE ResBlock tail); px * Cout must be 256, or Cout = 128 at px 1 (512 x 128 tile)."""
    _dev(x, "conv3x3_rmsnorm(x)", torch.bfloat16)
    _dev(w_packed, "conv3x3_rmsnorm(w)", torch.bfloat16)
    _dev(norm_w, "conv3x3_rmsnorm(norm_w)", torch.bfloat16)
    _dev(res, "conv3x3_rmsnorm(res)", torch.bfloat16)
    x, res = x.contiguous(), res.contiguous()
    B, H, W, Cin = x.shape
    N = w_packed.shape[0]
    if (N != 256 and not (N == 128 and px == 1)) or w_packed.shape[1] != 3 * (px + 2) * Cin \
            or res.shape != (B, H, W, N // px):
        raise ValueError(f"conv3x3_rmsnorm: packed weight {tuple(w_packed.shape)} / res {tuple(res.shape)} do not "
                         f"match x {tuple(x.shape)}, px={px} (px * Cout must be 256, or 128 at px 1)")
    for t, nm in ((bias, "bias"), (norm_b, "norm_b")):
        if t is not None:
            _dev(t, f"conv3x3_rmsnorm({nm})", torch.bfloat16)
    out = torch.empty_like(res)
    e0 = OpTimer.begin()
    _lib.call("eggroll_conv3x3_rmsnorm_nhwc_sel", x.data_ptr(), w_packed.data_ptr(), _p(bias), B, H, W, Cin, N, px,
              float(eps), norm_w.data_ptr(), _p(norm_b), res.data_ptr(), out.data_ptr(), int(kernel),
              _stream(x.device))
    OpTimer.end(e0, "conv3x3", 2.0 * (x.numel() + 2 * out.numel()), f"{tuple(x.shape)}->{N // px} px{px} +norm",
                flops=2.0 * B * H * W * (N // px) * 9 * Cin)
    return out


def bias_act_(y: torch.Tensor, bias: torch.Tensor, act: Optional[str]) -> torch.Tensor:
    """y = act(y + bias) in place over the last (channel) dim of a contiguous bf16 tensor."""
    _dev(y, "bias_act(y)", torch.bfloat16)
    _dev(bias, "bias_act(bias)", torch.bfloat16)
    if not y.is_contiguous() or bias.numel() != y.shape[-1]:
        raise ValueError("bias_act: y must be contiguous with bias over its last dim")
    C = y.shape[-1]
    e0 = OpTimer.begin()
    _lib.call("eggroll_bias_act", y.data_ptr(), bias.data_ptr(), y.numel() // C, C, ACT[act], _stream(y.device))
    OpTimer.end(e0, "bias_act", 4.0 * y.numel(), f"{tuple(y.shape)}")
    return y


# eggroll_cross_attention_sel's kernel form: 0 automatic (online two-half softmax), 1 two-pass, 2 online.
# The product runs 0; tests/test_gpu_rank_fidelity_fullsize.py scores the same epochs through 1 and 2.
XATTN_VARIANT = 0


def cross_attention(q: torch.Tensor, k: torch.Tensor, v: torch.Tensor, B: int, N: int, heads: int, head_dim: int,
                    L: int, scale: float, bias: Optional[torch.Tensor] = None, enc_index: Optional[torch.Tensor] = None,
                    out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Sana attn2 softmax cross-attention on MFMA (eggroll_cross_attention).  q: [B*N, >= heads*hd] bf16
    rows; k, v: [U*L, >= heads*hd] bf16 caption rows; bias [U, L] bf16 (additive mask) or None;
    enc_index [B] int (image -> caption row) or None.  Returns [B*N, heads*hd] bf16."""
    for t, nm in ((q, "q"), (k, "k"), (v, "v")):
        if t.device.type != "cuda" or t.dtype != torch.bfloat16 or t.stride(-1) != 1:
            raise _lib.EggrollError(f"cross_attention({nm}): expected a bf16 device view with unit inner stride")
    if k.stride(0) != v.stride(0):
        raise ValueError("cross_attention: k / v must share a row stride")
    if (k.shape[0] != v.shape[0] or k.shape[0] % L or k.shape[0] == 0 or min(k.shape[1], v.shape[1]) < heads * head_dim):
        raise ValueError(f"cross_attention: k / v {tuple(k.shape)} / {tuple(v.shape)} are not [U*L, >= heads*hd] "
                         f"with L={L}")
    U = k.shape[0] // L
    if q.shape[0] < B * N or q.shape[1] < heads * head_dim:
        raise ValueError(f"cross_attention: q {tuple(q.shape)} has fewer than B*N={B * N} rows of heads*hd")
    if out is None:
        out = torch.empty((B * N, heads * head_dim), dtype=torch.bfloat16, device=q.device)
    if bias is not None:
        _dev(bias, "cross_attention(bias)", torch.bfloat16)
        if tuple(bias.shape) != (U, L):
            raise ValueError(f"cross_attention: bias {tuple(bias.shape)} must be [U, L] = [{U}, {L}]")
    ei = None
    if enc_index is not None:
        if enc_index.numel() != B:
            raise ValueError(f"cross_attention: enc_index has {enc_index.numel()} entries, expected B={B}")
        if enc_index.device.type == "cpu" and B and (int(enc_index.min()) < 0 or int(enc_index.max()) >= U):
            raise ValueError(f"cross_attention: enc_index outside [0, {U})")
        # a device-resident enc_index is range-checked in the kernel (out-of-range images come out NaN)
        ei = enc_index.to(device=q.device, dtype=torch.int32).contiguous()
    elif U < B:
        raise ValueError(f"cross_attention: {U} caption rows for B={B} images without enc_index")
    e0 = OpTimer.begin()
    _lib.call("eggroll_cross_attention_sel", q.data_ptr(), q.stride(0), k.data_ptr(), v.data_ptr(), k.stride(0),
              _p(bias), _p(ei), B, N, heads, head_dim, L, U, float(scale), out.data_ptr(), out.stride(0),
              int(XATTN_VARIANT), _stream(q.device))
    OpTimer.end(e0, "cross_attention", 2.0 * (2 * B * N * heads * head_dim + 2 * k.shape[0] * heads * head_dim),
                f"B{B} N{N} L{L}")
    return out


def flash_attention(q: torch.Tensor, k: torch.Tensor, v: torch.Tensor, scale: float,
                    out: Optional[torch.Tensor] = None, qf: int = 0) -> torch.Tensor:
    """softmax(scale * q k^T) v on MFMA (eggroll_flash_attention), head dim 128, no mask.  q [B, Nq, H, 128],
    k / v [B, Lk, H, 128] bf16 views with unit inner stride and heads 128 apart (batch and row strides
    free: a KV-cache slice is read in place).  Returns [B, Nq, H, 128] bf16 (or writes `out`)."""
    for t, nm in ((q, "q"), (k, "k"), (v, "v")):
        if t.device.type != "cuda" or t.dtype != torch.bfloat16 or t.dim() != 4 or t.stride(3) != 1 or t.stride(2) != 128:
            raise _lib.EggrollError(f"flash_attention({nm}): expected a bf16 device view [B, S, H, 128] with heads "
                                    f"128 apart, got {tuple(t.shape)} / {t.stride()}")
    B, Nq, H, D = q.shape
    if D != 128 or k.shape[0] != B or v.shape[0] != B or k.shape[2] != H or v.shape[2] != H or k.shape[1] != v.shape[1]:
        raise ValueError(f"flash_attention: q {tuple(q.shape)}, k {tuple(k.shape)}, v {tuple(v.shape)}")
    if out is None:
        out = torch.empty((B, Nq, H, D), dtype=torch.bfloat16, device=q.device)
    elif out.dtype != torch.bfloat16 or out.stride(3) != 1 or out.stride(2) != 128 or tuple(out.shape) != (B, Nq, H, D):
        raise ValueError("flash_attention: out must be a bf16 [B, Nq, H, 128] view with heads 128 apart")
    e0 = OpTimer.begin()
    _lib.call("eggroll_flash_attention_sel", q.data_ptr(), q.stride(0), q.stride(1), k.data_ptr(), k.stride(0),
              k.stride(1), v.data_ptr(), v.stride(0), v.stride(1), B, H, Nq, k.shape[1], 128, float(scale), out.data_ptr(),
              out.stride(0), out.stride(1), int(qf), _stream(q.device))
    OpTimer.end(e0, "flash_attention", 2.0 * B * H * 128 * (2 * Nq + 2 * k.shape[1]), f"B{B} Nq{Nq} Lk{k.shape[1]} h{H}",
                flops=4.0 * B * H * Nq * k.shape[1] * 128)
    return out


def group_norm_nhwc(x: torch.Tensor, groups: int, w: torch.Tensor, b: torch.Tensor, eps: float,
                    silu: bool = False) -> torch.Tensor:
    """GroupNorm over an NHWC bf16 tensor [B, H, W, C] (+ SiLU), fp32 statistics
    (eggroll_group_norm_nhwc).  Returns a new contiguous [B, H, W, C] bf16 tensor."""
    _dev(x, "group_norm(x)", torch.bfloat16)
    _dev(w, "group_norm(w)", torch.bfloat16)
    _dev(b, "group_norm(b)", torch.bfloat16)
    B, C = x.shape[0], x.shape[-1]
    HW = x.numel() // max(B * C, 1)
    out = torch.empty_like(x)
    nb = int(_lib.load().eggroll_group_norm_workspace_bytes(B, HW, C, groups))
    ws = torch.empty(max(1, -(-nb // 8)), dtype=torch.float64, device=x.device)
    e0 = OpTimer.begin()
    _lib.call("eggroll_group_norm_nhwc", x.data_ptr(), B, HW, C, int(groups), float(eps), w.data_ptr(), b.data_ptr(),
              int(bool(silu)), out.data_ptr(), ws.data_ptr(), _stream(x.device))
    OpTimer.end(e0, f"group_norm(C={C})", 6.0 * x.numel(), f"B{B} HW{HW}")
    return out
