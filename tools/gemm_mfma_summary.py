"""MFMA-busy fraction of the LoRA GEMM kernels from one rocprofv3 --pmc pass (SQ_VALU_MFMA_BUSY_CYCLES,
SQ_INSTS_VALU_MFMA_MOPS_BF16, SQ_BUSY_CYCLES, GRBM_GUI_ACTIVE) + one --kernel-trace pass for durations.

  mfma_busy = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE x 128)
SQ_VALU_MFMA_BUSY_CYCLES sums SIMD-cycles with an MFMA executing over all SIMDs (MI355X_MICROARCH.md: 32 per
32x32x16 bf16 MFMA, 16 per 16x16x32); GRBM_GUI_ACTIVE sums the busy cycles of the 8 XCDs, each with 32 CUs x
4 SIMDs = 128 SIMDs, so GUI x 128 is the SIMD-cycles available.  clock = GRBM_GUI_ACTIVE / 8 / duration.
Also: the same fraction against the 2.5-PF vendor peak's clock (2.4 GHz) — MFMA cycles / (duration x 2.4 GHz
x 1024) — and the MFMA count implied by the counter vs the algorithmic one (2MNK / (2 x 16 x 16 x 32) + the
LoRA addend k-step).
usage: python tools/gemm_mfma_summary.py <pmc_dir> <trace_dir> [--out profiles/pmc_lora_gemm_mfma.json]"""
import argparse
import csv
import json
from collections import defaultdict
from pathlib import Path

ap = argparse.ArgumentParser()
ap.add_argument("pmc_dir")
ap.add_argument("trace_dir")
ap.add_argument("--out", default="profiles/pmc_lora_gemm_mfma.json")
A = ap.parse_args()


def find(d, pat):
    fs = sorted(Path(d).rglob(pat))
    if not fs:
        raise SystemExit(f"no {pat} under {d}")
    return fs[0]


def short(name):
    return name.split("(")[0].replace("void ", "").replace("eggroll::", "")


ctr = defaultdict(lambda: defaultdict(list))
for r in csv.DictReader(open(find(A.pmc_dir, "*counter_collection.csv"))):
    if "k_lora_gemm" not in r["Kernel_Name"]:
        continue
    ctr[short(r["Kernel_Name"])][r["Counter_Name"]].append(float(r["Counter_Value"]))
dur = defaultdict(list)
for r in csv.DictReader(open(find(A.trace_dir, "*kernel_trace.csv"))):
    if "k_lora_gemm" not in r["Kernel_Name"]:
        continue
    dur[short(r["Kernel_Name"])].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9)
M, N, Kd, r_ = 131072, 2240, 2240, 2
n_mfma_alg = 2.0 * M * N * Kd / (2 * 16 * 16 * 32)
out = {"shape": f"{M}x{N}x{Kd}, LoRA r {r_}, 8 members (Sana attn1 / attn2 projections, the bench's roofline kernel)",
       "method": "rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_BUSY_CYCLES GRBM_GUI_ACTIVE "
                 "(one pass) + --kernel-trace (durations), tools/gemm_mfma_driver.py", "kernels": {}}
for k, c in ctr.items():
    n = len(c["GRBM_GUI_ACTIVE"])
    gui = sum(c["GRBM_GUI_ACTIVE"]) / n
    busy = sum(c["SQ_VALU_MFMA_BUSY_CYCLES"]) / n
    mops = sum(c.get("SQ_INSTS_VALU_MFMA_MOPS_BF16", [0.0])) / n
    d = sorted(dur.get(k, [float("nan")]))
    t = d[len(d) // 2]
    clock = gui / 8 / t
    out["kernels"][k] = {
        "launches": n, "duration_us_median": t * 1e6, "clock_GHz": clock / 1e9,
        "mfma_busy_frac": busy / (gui * 128.0),
        "mfma_busy_frac_at_2.4GHz": busy / (t * 2.4e9 * 1024.0),
        "tflops": 2.0 * M * N * Kd * (1 + r_ / Kd) / t / 1e12,
        "mfma_busy_cycles": busy, "mfma_per_launch_from_busy_cycles": busy / 16.0,
        "mfma_per_launch_algorithmic": n_mfma_alg, "mfma_mops_bf16": mops,
    }
print(json.dumps(out, indent=1))
Path(A.out).write_text(json.dumps(out, indent=1))
