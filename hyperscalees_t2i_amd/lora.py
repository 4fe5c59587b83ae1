"""Population-aware LoRA linear — the drop-in for PEFT `lora.Linear` on the ES hot path.

Reference: PEFT LoRA injected by `get_peft_model(transformer, LoraConfig(r, alpha, dropout,
target_modules))` (es_backend.py:193-200); forward `y = base(x) + lora_B(lora_A(dropout(x))) *
alpha/r` with `lora_A.weight [r, in]`, `lora_B.weight [out, r]` (peft.tuners.lora.layer.Linear;
third-party, unpinned, not vendored — the formula is restated, see oracle.ref_lora_linear).

Two modes:
  * single-member (reference semantics): uses this module's own lora_A / lora_B parameters,
    i.e. whatever `unflatten_to_params` last wrote into them;
  * population (engine): a shared `PopulationContext` holds theta_pop [n_members, D] (fp32,
    one perturbed theta_k per member, written by the perturb kernel) and the rows of x are
    member-major; one eggroll_lora_linear_pop call evaluates every member, reading the frozen
    base weight through LDS once per tile for all members.
The base weight / bias are frozen bf16 (requires_grad=False, like PEFT's base_layer), so
`get_trainable_params_and_shapes` sees exactly (lora_A, lora_B) per layer in module order —
the reference theta layout (utills.py:141-152).
"""
from __future__ import annotations

import math
from dataclasses import dataclass
from typing import Dict, Iterable, List, Optional, Sequence

import torch
from torch import nn

from . import kernels as K


# Elementwise ops fused into GEMM epilogues (residual adds, gated residuals, the GLUMBConv SiLU).
# The fused and unfused forms run the same kernels and are bit-identical
# (tests/test_gpu_engine.py::test_fused_epilogues_bit_identical); False keeps every GEMM output
# materialised (per-linear captures in the fp32 drift test).
FUSE_EPILOGUES = True
# GLUMBConv's SiLU in the inverted conv's GEMM epilogue (True) or in the depthwise conv's staging (False,
# the default since round 5: the same bits, 1.2-3.5 % faster per GLUMBConv, profiles/r09q_silu_placement.log)
SILU_IN_GEMM = False


# bytes of one GEMM operand the kernels can address (32-bit buffer offsets); larger X runs in row chunks
GEMM_OPERAND_LIMIT = 1 << 31


@dataclass
class PopulationContext:
    theta_pop: Optional[torch.Tensor] = None  # [n_members, ld] fp32 (perturbed theta per member)
    n_members: int = 1
    T_ws: Optional[torch.Tensor] = None       # reusable fp32 workspace for T = X A_k^T
    multi_ws: Optional[torch.Tensor] = None   # T of the linears sharing one input (shared_projection)

    def workspace(self, numel: int, device) -> torch.Tensor:
        if self.T_ws is None or self.T_ws.numel() < numel or self.T_ws.device != torch.device(device):
            self.T_ws = torch.empty(max(numel, 1), dtype=torch.float32, device=device)
        return self.T_ws

    def multi_workspace(self, numel: int, device) -> torch.Tensor:
        if self.multi_ws is None or self.multi_ws.numel() < numel or self.multi_ws.device != torch.device(device):
            self.multi_ws = torch.empty(max(numel, 1), dtype=torch.float32, device=device)
        return self.multi_ws[:numel]


class GemmTimer:
    """Opt-in live timing of every population LoRA linear with HIP events recorded on the launching
    stream (bench.py's roofline leg).  The product path is kept — fused epilogues (the fp32 residual
    stream's res32 / gated32, bf16 res / gated, SiLU / GELU) and the shared projections included — but
    each linear's projection (k_lora_project, HBM-bound) and its GEMM + LoRA / op epilogue (MFMA-bound)
    are launched as their two kernels with an event between them (the linear_pop[_epi] C calls run the
    same two launches back to back: eggroll_lora_gemm_epi_sel is the second on its own), so each kernel's
    duration is its own — the figure rocprof reports per kernel.
    records: (e0 | None, e1, e2, M, N, K, r, rows_per_member, epi) — e0..e1 the projection (None when the
    shared projection made T), e1..e2 the GEMM; proj_records: (e0, e1, M, K, n_linears, r) of the
    shared projections."""

    active = False
    records: List[tuple] = []
    proj_records: List[tuple] = []

    @classmethod
    def reset(cls, active: bool):
        cls.active, cls.records, cls.proj_records = active, [], []

    @staticmethod
    def epilogue_bytes(M: int, N: int, epi: Optional[str]) -> float:
        """HBM bytes an epilogue op adds to the bf16 y write: fp32 stream read + write (+ its bf16 shadow)
        for res32 / gated32, the bf16 residual / multiplicand read for res / gated / mul."""
        if epi in ("res32", "gated32"):
            return 10.0 * M * N
        if epi in ("res", "gated", "mul"):
            return 2.0 * M * N
        return 0.0

    @classmethod
    def summary(cls) -> Dict[str, Dict[str, float]]:
        """Per GEMM kernel variant as rocprof names them (k_lora_gemm8<r> / k_lora_gemm8n<r> = the 8-phase
        256x256 / 256x320 tiles, k_lora_gemm<r,Tile<128>>; ",epi" = the fused op code of
        kernels.EPI) and "all": launches, total / avg kernel time, algorithmic FLOP = 2MNK (base) + 2MNr
        (rank-r LoRA expansion in the epilogue), the epilogue op's HBM bytes.  "k_lora_project<r>" /
        "k_lora_project_multi": the projection pre-passes, algorithmic bytes = X (2MK) + T (4Mr per linear)
        + the members' A rows (4 n_k r K per linear)."""
        torch.cuda.synchronize()
        out: Dict[str, Dict[str, float]] = {}
        for e0, e1, e2, M, N, Kd, r, rpm, epi in cls.records:
            t = K.gemm_tile_for(M, N, r, rpm, epi)
            code = K.EPI[epi]
            name = {8: f"k_lora_gemm8<{r},{code}>", 10: f"k_lora_gemm8n<{r},{code}>"}.get(t, f"k_lora_gemm<{r},Tile<{t}>>")
            ms = e1.elapsed_time(e2)
            fl = 2.0 * M * N * Kd + 2.0 * M * N * r
            for key in (name, "all"):
                d = out.setdefault(key, {"launches": 0, "total_ms": 0.0, "flops": 0.0, "epi_bytes": 0.0})
                d["launches"] += 1
                d["total_ms"] += ms
                d["flops"] += fl
                d["epi_bytes"] += cls.epilogue_bytes(M, N, epi)
                if key != "all":
                    d["shape"] = f"{M}x{N}x{Kd}"
            if e0 is not None:
                d = out.setdefault(f"k_lora_project<{r}>", {"launches": 0, "total_ms": 0.0, "bytes": 0.0})
                d["launches"] += 1
                d["total_ms"] += e0.elapsed_time(e1)
                d["bytes"] += 2.0 * M * Kd + 4.0 * M * r + 4.0 * (-(-M // rpm)) * r * Kd
        for e0, e1, M, Kd, nl, r in cls.proj_records:
            d = out.setdefault("k_lora_project_multi", {"launches": 0, "total_ms": 0.0, "bytes": 0.0})
            d["launches"] += 1
            d["total_ms"] += e0.elapsed_time(e1)
            d["bytes"] += 2.0 * M * Kd + nl * 4.0 * M * r
        for d in out.values():
            d["avg_us"] = 1e3 * d["total_ms"] / d["launches"]
            if "flops" in d:
                d["tflops"] = d["flops"] / (d["total_ms"] * 1e9) if d["total_ms"] > 0 else float("nan")
            else:
                d["GBps"] = d["bytes"] / (d["total_ms"] * 1e6) if d["total_ms"] > 0 else float("nan")
        return out

    @classmethod
    def events(cls, n: int):
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(n)]
        ev[0].record()
        return ev


class _Weight(nn.Module):
    """Holder so parameter names read `...lora_A.weight` / `...lora_B.weight` (PEFT naming)."""

    def __init__(self, shape):
        super().__init__()
        self.weight = nn.Parameter(torch.zeros(*shape, dtype=torch.float32))


class LoRALinear(nn.Module):
    def __init__(self, in_features: int, out_features: int, bias: bool = True, r: int = 2, alpha: float = 8.0,
                 lora: bool = True):
        super().__init__()
        self.in_features, self.out_features = in_features, out_features
        self.weight = nn.Parameter(torch.empty(out_features, in_features, dtype=torch.bfloat16), requires_grad=False)
        self.bias = (nn.Parameter(torch.zeros(out_features, dtype=torch.bfloat16), requires_grad=False)
                     if bias else None)
        self.r = r if lora else 0
        self.scale = float(alpha) / r if lora else 0.0
        if lora:
            self.lora_A = _Weight((r, in_features))
            self.lora_B = _Weight((out_features, r))
        self.ctx: Optional[PopulationContext] = None
        # plain (r = 0) GEMMs with at most this many rows go to the vendor library (F.linear -> hipBLASLt),
        # which splits K for short, wide problems; 0 = never (set per model: tools/small_m_gemm_probe.py)
        self.lib_small_m = 0
        self.theta_off_A = -1  # element offsets of lora_A / lora_B inside theta (set by bind_theta_layout)
        self.theta_off_B = -1

    def reset_lora(self, gen: Optional[torch.Generator] = None, b_std: float = 0.0):
        """PEFT default init: A ~ kaiming_uniform(a=sqrt(5)), B = 0 (b_std > 0: N(0, b_std), used by
        the benchmark so the LoRA path carries signal — SURVEY §8d)."""
        if not self.r:
            return
        bound = 1.0 / math.sqrt(self.in_features)  # kaiming_uniform_(a=sqrt(5)) on fan_in
        with torch.no_grad():
            self.lora_A.weight.uniform_(-bound, bound, generator=gen)
            if b_std > 0:
                self.lora_B.weight.normal_(0.0, b_std, generator=gen)
            else:
                self.lora_B.weight.zero_()

    def forward(self, x: torch.Tensor, epi: Optional[str] = None, res: Optional[torch.Tensor] = None,
                gate: Optional[torch.Tensor] = None, rows_per_group: int = 1,
                T: Optional[torch.Tensor] = None, shadow: Optional[torch.Tensor] = None) -> torch.Tensor:
        """epi (optional): an elementwise op on the output, fused into the GEMM epilogue on the
        population path (kernels.lora_linear_pop_epi): "res" -> res + y, "gated" -> res + gate[g] * y,
        "mul" -> res * y, written into `res` in place and returned; "res32" / "gated32": the same on an fp32 residual
        stream `res` (gate fp32), `shadow` (optional bf16) receiving bf16(res).  T (optional, population
        path): this linear's X A_k^T already computed by shared_projection — only the GEMM + LoRA
        epilogue run here."""
        shp = x.shape
        x2 = x.reshape(-1, shp[-1])
        if x2.dtype != torch.bfloat16:
            x2 = x2.to(torch.bfloat16)
        x2 = x2.contiguous()
        M = x2.shape[0]
        ctx = self.ctx
        if M * self.in_features * 2 >= GEMM_OPERAND_LIMIT:   # the GEMMs address X with 32-bit buffer offsets
            return self._forward_chunked(x2, shp, epi, res, gate, rows_per_group, T, shadow)
        if epi in ("silu", "gelu"):   # silu / gelu(tanh) of the bf16-rounded output, in the GEMM epilogue where it applies
            if (FUSE_EPILOGUES and ctx is not None and ctx.theta_pop is not None and self.r <= 2
                    and M % ctx.n_members == 0 and (self.r == 0 or M // ctx.n_members >= 256)
                    and self.in_features % 64 == 0):
                rpm = M // ctx.n_members
                ws = ctx.workspace(K.lora_workspace_numel(M, self.in_features, self.r, rpm), x2.device) if self.r else None
                if GemmTimer.active and self.r:
                    y = self._timed_epi(x2, ctx.theta_pop, ws, rpm, epi)
                else:
                    y = K.lora_linear_pop_epi(x2, self.weight, self.bias, ctx.theta_pop if self.r else None,
                                              self.theta_off_A, self.theta_off_B, self.r, self.scale, rpm, epi, T_ws=ws)
            elif epi == "silu":
                y = torch.nn.functional.silu(self.forward(x).view(M, self.out_features))
            else:
                y = torch.nn.functional.gelu(self.forward(x).view(M, self.out_features), approximate="tanh")
            return y.view(*shp[:-1], self.out_features)
        if epi is not None:
            res2 = res.view(M, self.out_features)
            sh2 = shadow.view(M, self.out_features) if shadow is not None else None
            if (FUSE_EPILOGUES and self.r and ctx is not None and ctx.theta_pop is not None and self.r <= 2
                    and M % ctx.n_members == 0 and M // ctx.n_members >= 256 and self.in_features % 64 == 0):
                rpm = M // ctx.n_members
                ws = ctx.workspace(K.lora_workspace_numel(M, self.in_features, self.r, rpm), x2.device)
                if GemmTimer.active:
                    self._timed_epi(x2, ctx.theta_pop, ws, rpm, epi, res=res2, gate=gate, rows_per_group=rows_per_group,
                                    out=sh2)
                else:
                    K.lora_linear_pop_epi(x2, self.weight, self.bias, ctx.theta_pop, self.theta_off_A, self.theta_off_B,
                                          self.r, self.scale, rpm, epi, res=res2, gate=gate,
                                          rows_per_group=rows_per_group, T_ws=ws, out=sh2)
                return res
            if (FUSE_EPILOGUES and not self.r and M >= max(4096, self.lib_small_m + 1)
                    and self.in_features % 64 == 0
                    and epi in ("res", "gated", "mul")):   # plain linear (no LoRA), epilogue fused (Infinity's proj / fc2)
                K.lora_linear_pop_epi(x2, self.weight, self.bias, None, 0, 0, 0, 0.0, M, epi, res=res2, gate=gate,
                                      rows_per_group=rows_per_group)
                return res
            y = self.forward(x).view(M, self.out_features)   # the same ops, unfused
            if epi == "res":
                res2.add_(y)
            elif epi == "mul":
                res2.mul_(y)
            elif epi == "gated":
                K.gated_residual_(res2, y, gate, rows_per_group=rows_per_group)
            elif epi in ("res32", "gated32"):
                K.gated_residual_f32_(res2, y, gate if epi == "gated32" else None, rows_per_group, shadow=sh2)
            else:
                raise ValueError(f"LoRALinear: epi {epi!r} unsupported")
            return res
        if self.r and ctx is not None and ctx.theta_pop is not None:
            if M % ctx.n_members:
                raise RuntimeError(f"{M} rows do not split over {ctx.n_members} members")
            rpm = M // ctx.n_members
            ws = ctx.workspace(K.lora_workspace_numel(M, self.in_features, self.r, rpm), x2.device)
            if T is not None:     # projection already done for the linears sharing this input
                ev = GemmTimer.events(2) if GemmTimer.active else None
                y = K.lora_gemm(x2, self.weight, self.bias, T, ctx.theta_pop, self.theta_off_B, self.r, self.scale,
                                rpm)
                if ev is not None:
                    ev[1].record()
                    GemmTimer.records.append((None, ev[0], ev[1], M, self.out_features, self.in_features, self.r, rpm,
                                              None))
            elif GemmTimer.active:  # the same two kernels as lora_linear_pop's unfused path, timed apart
                ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
                T = ws[: M * self.r].view(M, self.r)
                ev[0].record()
                K.lora_project(x2, ctx.theta_pop, self.theta_off_A, self.r, rpm, out=T)
                ev[1].record()
                y = K.lora_gemm(x2, self.weight, self.bias, T, ctx.theta_pop, self.theta_off_B, self.r, self.scale,
                                rpm)
                ev[2].record()
                GemmTimer.records.append((*ev, M, self.out_features, self.in_features, self.r, rpm, None))
            else:  # projection T = X A_k^T + GEMM + LoRA epilogue (one fused kernel when eligible)
                y = K.lora_linear_pop(x2, self.weight, self.bias, ctx.theta_pop, self.theta_off_A, self.theta_off_B,
                                      self.r, self.scale, rpm, T_ws=ws)
        elif self.r:
            # single member: this module's own (unflattened) lora_A / lora_B
            A = self.lora_A.weight.detach()
            B = self.lora_B.weight.detach()
            if A.device != x2.device:
                raise RuntimeError("LoRA parameters and input on different devices")
            y = K.lora_linear_pop(x2, self.weight, self.bias, None, 0, 0, 0, 0.0, M)
            T = K.lora_project(x2, A.contiguous().view(1, -1), 0, self.r, M)
            K.lora_expand(T, B.contiguous().view(1, -1), 0, self.r, self.scale, M, y)
        elif M <= self.lib_small_m:
            y = torch.nn.functional.linear(x2, self.weight, self.bias)
        else:
            y = K.lora_linear_pop(x2, self.weight, self.bias, None, 0, 0, 0, 0.0, M)
        return y.view(*shp[:-1], self.out_features)


    def _timed_epi(self, x2, theta_pop, ws, rpm, epi, res=None, gate=None, rows_per_group=1, out=None):
        """lora_linear_pop_epi as its two launches with HIP events around each (GemmTimer): the projection,
        then the epilogue GEMM on that T — the same kernels and bits as the fused call."""
        M = x2.shape[0]
        T = ws[: M * self.r].view(M, self.r)
        ev = GemmTimer.events(3)
        K.lora_project(x2, theta_pop, self.theta_off_A, self.r, rpm, out=T)
        ev[1].record()
        y = K.lora_gemm_epi(x2, self.weight, self.bias, T, theta_pop, self.theta_off_B, self.r, self.scale, rpm, epi,
                            res=res, gate=gate, rows_per_group=rows_per_group, out=out)
        ev[2].record()
        GemmTimer.records.append((*ev, M, self.out_features, self.in_features, self.r, rpm, epi))
        return y

    def _forward_chunked(self, x2, shp, epi, res, gate, rows_per_group, T, shadow):
        """forward() over row chunks whose X stays under 2 GiB: whole members per chunk on the population
        path (theta_pop rows sliced alongside), any 256-row multiple otherwise."""
        M, ctx = x2.shape[0], self.ctx
        limit = max(256, (GEMM_OPERAND_LIMIT // (2 * self.in_features) - 1) // 256 * 256)
        pop = self.r and ctx is not None and ctx.theta_pop is not None
        if pop:
            n = ctx.n_members
            if M % n:
                raise RuntimeError(f"{M} rows do not split over {n} members")
            rpm = M // n
            if rpm > limit:
                raise RuntimeError(f"one member's {rpm} x {self.in_features} rows exceed the GEMM's 2 GiB operand")
            per = limit // rpm
            bounds = [(k0 * rpm, min(k0 + per, n) * rpm, k0, min(k0 + per, n)) for k0 in range(0, n, per)]
        else:
            bounds = [(r0, min(r0 + limit, M), 0, 0) for r0 in range(0, M, limit)]
        outs = []
        try:
            for r0, r1, k0, k1 in bounds:
                if pop:
                    sub = PopulationContext()
                    sub.theta_pop, sub.n_members, sub.T_ws, sub.multi_ws = ctx.theta_pop[k0:k1], k1 - k0, ctx.T_ws, ctx.multi_ws
                    self.ctx = sub
                g = None
                if gate is not None:
                    if r0 % rows_per_group:
                        raise RuntimeError("row chunk does not start on a gate group boundary")
                    g = gate[r0 // rows_per_group:]
                rr = res.view(M, self.out_features)[r0:r1] if res is not None else None
                sh = shadow.view(M, self.out_features)[r0:r1] if shadow is not None else None
                outs.append(self.forward(x2[r0:r1], epi=epi, res=rr, gate=g, rows_per_group=rows_per_group,
                                         T=T[r0:r1] if T is not None else None, shadow=sh))
                if pop:
                    ctx.T_ws, ctx.multi_ws = sub.T_ws, sub.multi_ws
        finally:
            self.ctx = ctx
        if res is not None and epi not in (None, "silu"):
            return res
        return torch.cat(outs).view(*shp[:-1], self.out_features)

    def _weight32(self) -> torch.Tensor:
        key = (self.weight._version, self.weight.data_ptr())
        if getattr(self, "_w32_key", None) != key:
            self._w32 = (self.weight.detach().float(), None if self.bias is None else self.bias.detach().float())
            self._w32_key = key
        return self._w32

    def forward_fp32(self, x: torch.Tensor) -> torch.Tensor:
        """The PEFT LoRA linear in fp32: y = x W^T + b (the library fp32 GEMM on an fp32 copy of the frozen
        weight) + s (x A_k^T) B_k^T (eggroll_lora_delta_f32, in place) with member k's factors from the
        population context (rows member-major) or this module's own lora_A / lora_B.  For the small-M
        linears whose outputs set a whole member's behaviour — the time / guidance embedding and AdaLN
        modulation, and proj_out (the transformer output the reference rounds to fp16 only): their bf16
        rounding was a measured source of member-differential error at sigma = 1e-2 (DESIGN §3.2,
        tools/drift_probe.py)."""
        shp = x.shape
        x2 = x.reshape(-1, shp[-1]).float().contiguous()
        M = x2.shape[0]
        W32, b32 = self._weight32()
        y = torch.nn.functional.linear(x2, W32, b32)
        ctx = self.ctx
        if self.r and ctx is not None and ctx.theta_pop is not None:
            n = ctx.n_members
            if M % n:
                raise RuntimeError(f"{M} rows do not split over {n} members")
            tp = ctx.theta_pop
            if FP32_DELTA_KERNEL and self.r <= LORA_DELTA_F32_MAX_R:
                K.lora_delta_f32(x2, tp[:, self.theta_off_A:], tp.stride(0), tp[:, self.theta_off_B:], tp.stride(0),
                                 self.r, self.scale, M // n, y)
            else:
                A = tp[:, self.theta_off_A:self.theta_off_A + self.r * self.in_features].view(n, self.r, -1)
                B = tp[:, self.theta_off_B:self.theta_off_B + self.out_features * self.r].view(n, self.out_features, -1)
                t = torch.bmm(x2.view(n, M // n, -1), A.transpose(1, 2))
                y = y + self.scale * torch.bmm(t, B.transpose(1, 2)).view(M, -1)
        elif self.r:
            A, B = self.lora_A.weight.detach().float().contiguous(), self.lora_B.weight.detach().float().contiguous()
            if self.r <= LORA_DELTA_F32_MAX_R:
                K.lora_delta_f32(x2, A, 0, B, 0, self.r, self.scale, max(M, 1), y)
            else:   # ranks above the kernel's register budget: the plain fp32 product
                y = y + self.scale * ((x2 @ A.t()) @ B.t())
        y = y.view(*shp[:-1], self.out_features)
        for hook in self._forward_hooks.values():   # forward hooks see this path like __call__ (activation capture)
            hook(self, (x,), y)
        return y


# LoRALinear.forward_fp32's population LoRA term on eggroll_lora_delta_f32 (True) or two torch bmm's (False, the
# round-4 form: A/B measurement only)
FP32_DELTA_KERNEL = True
# eggroll_lora_delta_f32 holds the r projections per row in registers: 1 <= r <= 8 (include/eggroll.h).  LoRA
# ranks above it (--sana_lora_r 16 etc.; the bf16 population GEMM takes r up to 16) use the two bmm's.
LORA_DELTA_F32_MAX_R = 8


# Linears that read the same input (Sana attn1 to_q / to_k / to_v, attn2 to_k / to_v) get their LoRA
# projections T_l = X A_{k,l}^T from ONE pass over X (kernels.lora_project_multi) instead of one pass
# per linear; False restores the per-linear projection (A/B measurement).
SHARED_PROJECTION = True


def shared_projection(mods: Sequence[LoRALinear], x: torch.Tensor) -> List[Optional[torch.Tensor]]:
    """[T_l] for mods on input x (population path), or [None] * len(mods) where it does not apply
    (single-member mode, LoRA off, GemmTimer's per-kernel timing, unsupported shapes)."""
    none = [None] * len(mods)
    ctx = mods[0].ctx if mods else None
    if (not SHARED_PROJECTION or ctx is None or ctx.theta_pop is None or len(mods) < 2
            or any(m.ctx is not ctx for m in mods)):
        return none
    r, Kd = mods[0].r, mods[0].in_features
    if (r == 0 or any(m.r != r or m.in_features != Kd for m in mods) or len(mods) * r > 8 or len(mods) > 4
            or Kd % 32 or Kd > 4096):
        return none
    x2 = x.reshape(-1, Kd)
    if x2.dtype != torch.bfloat16 or not x2.is_contiguous() or x2.data_ptr() % 16 or ctx.theta_pop.data_ptr() % 16:
        return none   # the multi-projection kernel issues 16-byte vector loads of X and theta_pop
    M = x2.shape[0]
    if M % ctx.n_members:
        raise RuntimeError(f"{M} rows do not split over {ctx.n_members} members")
    ws = ctx.multi_workspace(len(mods) * M * r, x2.device).view(len(mods), M, r)
    ev = GemmTimer.events(2) if GemmTimer.active else None
    K.lora_project_multi(x2, ctx.theta_pop, [m.theta_off_A for m in mods], r, M // ctx.n_members, out=ws)
    if ev is not None:
        ev[1].record()
        GemmTimer.proj_records.append((ev[0], ev[1], M, Kd, len(mods), r))
    return [ws[i] for i in range(len(mods))]


def lora_modules(model: nn.Module) -> List[LoRALinear]:
    return [m for m in model.modules() if isinstance(m, LoRALinear) and m.r]


def bind_theta_layout(model: nn.Module, base: int = 0) -> Dict[str, int]:
    """Record each LoRA module's (lora_A, lora_B) offsets inside theta, following the trainable
    parameter order of model.parameters() (utills.py:141-152).  base: where this model's parameters
    start inside theta (a second LoRA'd model after the first, e.g. Z-Image's VAE decoder after its
    transformer, es_backend.py:613-618).  Returns {param_name: offset}."""
    offs, off = {}, int(base)
    by_param = {}
    for name, p in model.named_parameters():
        if p.requires_grad:
            offs[name] = off
            by_param[id(p)] = off
            off += p.numel()
    for m in lora_modules(model):
        m.theta_off_A = by_param[id(m.lora_A.weight)]
        m.theta_off_B = by_param[id(m.lora_B.weight)]
        if m.theta_off_A % 4:
            raise RuntimeError("lora_A offset inside theta must be 16-byte aligned for the project kernel")
    return offs


def set_population(model: nn.Module, ctx: Optional[PopulationContext]) -> None:
    for m in lora_modules(model):
        m.ctx = ctx
