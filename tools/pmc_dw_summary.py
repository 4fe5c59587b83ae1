"""Per-shape summary of tools/pmc_dw.sh: duration (kernel trace), instruction mix and wait fractions,
HBM bytes (FETCH_SIZE x 2 on gfx950, MI355X_MICROARCH.md) vs the algorithmic bytes, VALU-issue
bound.  Launches are matched to shapes by grid size.
usage: python tools/pmc_dw_summary.py <tag> [--out profiles/<file>.json]"""
import argparse
import csv
import json
import math
from collections import defaultdict
from pathlib import Path

ap = argparse.ArgumentParser()
ap.add_argument("tag")
ap.add_argument("--out", default=None)
A = ap.parse_args()
G = Path("gpurun_out")
SHAPES = ((128, 32, 32, 11200, 3, False, True), (8, 128, 128, 4096, 3, False, True),
          (8, 64, 64, 8192, 3, True, True), (8, 128, 128, 1536, 5, False, False))


def grid(B, H, W, C, glu):
    cout = C // 2 if glu else C
    return B * math.ceil(H / 8) * math.ceil(W / 32) * (cout // 32) * 256


def alg_bytes(B, H, W, C, ks, glu):
    return B * H * W * C * 2 + B * H * W * (C // 2 if glu else C) * 2


def rows(p, f):
    fs = sorted((G / f"{A.tag}_{p}").rglob(f))
    if not fs:
        raise SystemExit(f"no {f} for pass {p}")
    return list(csv.DictReader(open(fs[0])))


key = {grid(B, H, W, C, glu): f"{B}x{H}x{W}x{C} ks{ks} pre{int(pre)} glu{int(glu)}{'' if glu else ' pw'}"
       for B, H, W, C, ks, pre, glu in SHAPES}
alg = {grid(B, H, W, C, glu): alg_bytes(B, H, W, C, ks, glu) for B, H, W, C, ks, pre, glu in SHAPES}
dur = defaultdict(list)
for r in rows("tr", "*kernel_trace.csv"):
    if "k_dwconv" not in r["Kernel_Name"]:
        continue
    dur[int(r["Grid_Size_X"])].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9)
ctr = defaultdict(lambda: defaultdict(list))
for p in ("p1", "p2", "p3", "p4"):
    for r in rows(p, "*counter_collection.csv"):
        ctr[int(r["Grid_Size"])][r["Counter_Name"]].append(float(r["Counter_Value"]))
out = {"method": "tools/pmc_dw.sh: rocprofv3 --kernel-trace + 4 --pmc passes over tools/dw_driver.py (3 launches "
                 "per shape); per-launch means", "shapes": {}}
for g, name in key.items():
    d = sorted(dur.get(g, [float("nan")]))
    t = d[len(d) // 2]
    c = {k: sum(v) / len(v) for k, v in ctr[g].items()}
    gui = c.get("GRBM_GUI_ACTIVE", float("nan"))
    clock = gui / 8 / t
    fetch = c.get("FETCH_SIZE", float("nan")) * 1024 * 2   # KiB; reports half the bytes on gfx950
    write = c.get("WRITE_SIZE", float("nan")) * 1024
    waves = c.get("SQ_WAVES", float("nan"))
    valu = c.get("SQ_INSTS_VALU", float("nan"))
    # VALU issue bound: every wave's VALU instructions on 1024 SIMDs, >= 1 cycle each (4 for wave64 fp32
    # non-packed on a 16-lane SIMD; packed / DPFP rates differ): the issue-cycle floor from SQ_ACTIVE_INST_VALU
    act_valu = c.get("SQ_ACTIVE_INST_VALU", float("nan"))
    out["shapes"][name] = {
        "launch_us": t * 1e6, "clock_GHz": clock / 1e9,
        "alg_bytes": alg[g], "alg_TBps": alg[g] / t / 1e12, "frac_hbm_alg": alg[g] / t / 8e12,
        "fetch_bytes": fetch, "write_bytes": write, "hbm_TBps": (fetch + write) / t / 1e12,
        "l2_hit": c.get("TCC_HIT_sum", 0) / max(1.0, c.get("TCC_HIT_sum", 0) + c.get("TCC_MISS_sum", 0)),
        "waves": waves, "valu_per_wave": valu / waves, "lds_per_wave": c.get("SQ_INSTS_LDS", 0) / waves,
        "salu_per_wave": c.get("SQ_INSTS_SALU", 0) / waves, "trans_per_wave": c.get("SQ_INSTS_VALU_TRANS_F32", 0) / waves,
        # SQ_ACTIVE_INST_VALU / SQ_BUSY_CYCLES: cycles (per SQ, x4 quad-cycles) with a VALU instruction in
        # flight; the fractions below are relative to the wave-cycles (SQ_WAVE_CYCLES) unless stated
        "valu_active_over_wave_cycles": act_valu / c.get("SQ_WAVE_CYCLES", float("nan")),
        "wait_any_over_wave_cycles": c.get("SQ_WAIT_ANY", 0) / c.get("SQ_WAVE_CYCLES", float("nan")),
        "wait_inst_any_over_wave_cycles": c.get("SQ_WAIT_INST_ANY", 0) / c.get("SQ_WAVE_CYCLES", float("nan")),
        "lds_active_over_wave_cycles": c.get("SQ_ACTIVE_INST_LDS", 0) / c.get("SQ_WAVE_CYCLES", float("nan")),
        "valu_thread_cycles_per_valu": c.get("SQ_THREAD_CYCLES_VALU", 0) / max(1.0, valu),
        "mean_waves_resident_per_cu": c.get("SQ_LEVEL_WAVES", 0) / max(1.0, c.get("SQ_WAVE_CYCLES", 1)) * 0,
        "lds_bank_conflict_per_wave": c.get("SQ_LDS_BANK_CONFLICT", 0) / waves,
        "vmem_rd_cycles_per_wave": c.get("SQ_INST_CYCLES_VMEM_RD", 0) / waves,
        "raw": c,
    }
txt = json.dumps(out, indent=1)
print(txt)
if A.out:
    Path(A.out).write_text(txt)
