"""VALU roofline of the seeded ES kernels from tools/pmc_es_valu.sh (one SQ pass + one kernel trace).

Launches are grouped by (kernel, grid size) — the two driver configurations have different grids.  Per group:
  clock        = GRBM_GUI_ACTIVE / 8 XCDs / duration
  valu_active  = SQ_ACTIVE_INST_VALU x 4 (quad-cycles) / (clock cycles x 1024 SIMDs): the share of SIMD-cycles
                 a wave spent issuing VALU work (quarter-rate multiplies and transcendentals included)
  valu_issue_2 = SQ_INSTS_VALU x 2 / (cycles x 1024): the same at the full-rate wave64 issue cost (2 cycles on
                 the 32-lane SIMD, MI355X_MICROARCH.md), i.e. a lower bound that counts every op as full rate
  valu_active_at_2.4GHz = the VALU-active SIMD-cycles over duration x 2.4 GHz x 1024: against the peak clock (the
                 GRBM window of a 15-30 us launch includes dispatch overhead, so its clock reads high: > 2.4 GHz)
usage: python tools/es_valu_summary.py <pmc_dir> <trace_dir> [--out profiles/pmc_es_seeded_valu.json]"""
import argparse
import csv
import json
from collections import defaultdict
from pathlib import Path

ap = argparse.ArgumentParser()
ap.add_argument("pmc_dir")
ap.add_argument("trace_dir")
ap.add_argument("--out", default="profiles/pmc_es_seeded_valu.json")
A = ap.parse_args()


def find(d, pat):
    fs = sorted(Path(d).rglob(pat))
    if not fs:
        raise SystemExit(f"no {pat} under {d}")
    return fs[0]


def key(r):
    return r["Kernel_Name"].split("(")[0].replace("void ", "").replace("eggroll::", ""), r.get("Grid_Size") or r.get("Grid_Size_X", "?")


ctr = defaultdict(lambda: defaultdict(list))
for r in csv.DictReader(open(find(A.pmc_dir, "*counter_collection.csv"))):
    ctr[key(r)][r["Counter_Name"]].append(float(r["Counter_Value"]))
dur = defaultdict(list)
for r in csv.DictReader(open(find(A.trace_dir, "*kernel_trace.csv"))):
    dur[key(r)].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9)

out = {"method": "rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VALU_TRANS_F32 SQ_ACTIVE_INST_VALU SQ_INSTS_SALU "
                 "SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE (one pass) + --kernel-trace, tools/es_valu_driver.py "
                 "(Sana theta layout: pop 64 / 8 local members at egg rank 1, pop 128 / 16 local at rank 4)",
       "groups": {}}
for (name, grid), c in sorted(ctr.items()):
    n = len(c["GRBM_GUI_ACTIVE"])
    d = sorted(dur.get((name, grid), []))
    if not d:
        continue
    t = d[len(d) // 2]
    cyc = sum(c["GRBM_GUI_ACTIVE"]) / n / 8
    insts = sum(c["SQ_INSTS_VALU"]) / n
    trans = sum(c.get("SQ_INSTS_VALU_TRANS_F32", [0.0])) / n
    act = sum(c["SQ_ACTIVE_INST_VALU"]) / n
    out["groups"][f"{name} grid {grid}"] = {
        "launches": n, "duration_us_median": round(t * 1e6, 3), "clock_GHz": round(cyc / t / 1e9, 3),
        "valu_insts": insts, "trans_insts": trans, "salu_insts": sum(c["SQ_INSTS_SALU"]) / n,
        "waves": sum(c["SQ_WAVES"]) / n,
        "valu_active": round(act * 4 / (cyc * 1024), 3),
        "valu_issue_2": round(insts * 2 / (cyc * 1024), 3),
        "valu_active_at_2.4GHz": round(act * 4 / (t * 2.4e9 * 1024), 3),
    }
print(json.dumps(out, indent=1))
Path(A.out).write_text(json.dumps(out, indent=1))
