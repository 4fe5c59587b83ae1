"""Per-kernel census of one Sana ES epoch from tools/pmc_epoch.sh: time (kernel trace, dispatches between
the two marker launches), and from the counter passes (same window) the VALU-issue fraction, the MFMA-busy
fraction and the HBM rate.
  valu_issue = SQ_INSTS_VALU x 4 cycles (wave64 on a 16-lane SIMD; MFMA and transcendental ops counted at
               4, so this under-counts their issue time) / (1024 SIMDs x kernel cycles)
  mfma_busy  = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE x 128)   (GUI sums the 8 XCDs' cycles)
  hbm        = (FETCH_SIZE x 2 [gfx950] + WRITE_SIZE) KiB / trace duration
Kernels are grouped by the name up to the argument list.
usage: python tools/pmc_epoch_summary.py <tag> [--top 40] [--out file.json]"""
import argparse
import csv
import json
from collections import defaultdict
from pathlib import Path

ap = argparse.ArgumentParser()
ap.add_argument("tag")
ap.add_argument("--top", type=int, default=40)
ap.add_argument("--out", default=None)
A = ap.parse_args()
G = Path("gpurun_out")


def short(n):
    n = n.replace("void ", "")
    if "(" in n:
        n = n[:n.index("(")]
    return n.replace("eggroll::", "")[:90]


def rows(p, f):
    fs = sorted((G / f"{A.tag}_{p}").rglob(f))
    if not fs:
        raise SystemExit(f"no {f} for pass {p}")
    return list(csv.DictReader(open(fs[0])))


def window(rs, key):
    rs.sort(key=lambda r: int(r[key]))
    m = [i for i, r in enumerate(rs) if "k_philox_words" in r["Kernel_Name"]]
    return rs[m[0] + 1:m[1]] if len(m) >= 2 else rs


tr = window(rows("tr", "*kernel_trace.csv"), "Start_Timestamp")
agg = defaultdict(lambda: {"n": 0, "us": 0.0})
for r in tr:
    a = agg[short(r["Kernel_Name"])]
    a["n"] += 1
    a["us"] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
ctr = defaultdict(lambda: defaultdict(float))
for p in ("p1", "p2", "p3"):
    # counter rows: one per (dispatch, counter); window by dispatch order
    rs = rows(p, "*counter_collection.csv")
    disp = {}
    for r in rs:
        disp.setdefault(int(r["Dispatch_Id"]), r["Kernel_Name"])
    order = sorted(disp)
    m = [d for d in order if "k_philox_words" in disp[d]]
    lo, hi = (m[0], m[1]) if len(m) >= 2 else (order[0] - 1, order[-1] + 1)
    for r in rs:
        d = int(r["Dispatch_Id"])
        if lo < d < hi:
            ctr[short(r["Kernel_Name"])][p + ":" + r["Counter_Name"]] += float(r["Counter_Value"])
tot = sum(a["us"] for a in agg.values())
out = {"epoch_kernel_busy_ms": tot / 1e3, "kernels": {}}
for k, a in sorted(agg.items(), key=lambda kv: -kv[1]["us"])[:A.top]:
    c = ctr.get(k, {})
    gui1 = c.get("p1:GRBM_GUI_ACTIVE", 0.0)
    cyc = gui1 / 8
    e = {"launches": a["n"], "ms": round(a["us"] / 1e3, 3), "share": round(a["us"] / tot, 4)}
    if cyc > 0:
        e["valu_per_wave"] = round(c.get("p1:SQ_INSTS_VALU", 0) / max(1.0, c.get("p1:SQ_WAVES", 0)), 1)
        e["valu_issue"] = round(c.get("p1:SQ_INSTS_VALU", 0) * 4 / 1024 / cyc, 3)
        e["trans_share"] = round(c.get("p1:SQ_INSTS_VALU_TRANS_F32", 0) / max(1.0, c.get("p1:SQ_INSTS_VALU", 0)), 3)
        e["mfma_busy"] = round(c.get("p1:SQ_VALU_MFMA_BUSY_CYCLES", 0) / (gui1 * 128), 3)
        e["clock_GHz_pmc"] = round(cyc / (a["us"] * 1e-6) / 1e9, 3)
    fb = c.get("p2:FETCH_SIZE", 0) * 1024 * 2
    wb = c.get("p3:WRITE_SIZE", 0) * 1024
    if fb or wb:
        e["hbm_TBps"] = round((fb + wb) / (a["us"] * 1e-6) / 1e12, 3)
        e["fetch_GB"] = round(fb / 1e9, 3)
        e["write_GB"] = round(wb / 1e9, 3)
        h, mi = c.get("p3:TCC_HIT_sum", 0), c.get("p3:TCC_MISS_sum", 0)
        e["l2_hit"] = round(h / max(1.0, h + mi), 3)
    out["kernels"][k] = e
txt = json.dumps(out, indent=1)
if A.out:
    Path(A.out).write_text(txt)
print(f"epoch kernel-busy {tot / 1e3:.1f} ms")
for k, e in out["kernels"].items():
    print(f"{e['ms']:8.2f} ms {e['share']:6.3f} {k[:60]:60s} " + " ".join(f"{x}={e[x]}" for x in
          ("valu_issue", "mfma_busy", "hbm_TBps", "l2_hit", "valu_per_wave", "trans_share", "clock_GHz_pmc") if x in e))
