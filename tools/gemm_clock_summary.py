"""Effective clock and busy fraction per kernel from a `rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT
--kernel-trace` run (tools/gemm_clock_driver.py): GRBM_GUI_ACTIVE is summed over the 8 XCDs, so
clock = GUI_ACTIVE / 8 / duration.  usage: python tools/gemm_clock_summary.py <rocprof out dir>"""
import collections
import csv
import json
import statistics
import sys
from pathlib import Path

d = Path(sys.argv[1])
cc = next(d.rglob("*counter_collection.csv"))
kt = next(d.rglob("*kernel_trace.csv"))
dur = {}
for r in csv.DictReader(open(kt)):
    dur[r["Dispatch_Id"]] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
ctr = collections.defaultdict(dict)
names = {}
for r in csv.DictReader(open(cc)):
    ctr[r["Dispatch_Id"]][r["Counter_Name"]] = float(r["Counter_Value"])
    names[r["Dispatch_Id"]] = r["Kernel_Name"].split("(")[0]
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for did, c in ctr.items():
    if did not in dur or "GRBM_GUI_ACTIVE" not in c:
        continue
    n = names[did]
    agg[n]["us"].append(dur[did] * 1e6)
    agg[n]["clock_GHz"].append(c["GRBM_GUI_ACTIVE"] / 8 / dur[did] / 1e9)
    if "GRBM_COUNT" in c:
        agg[n]["gui_active_frac"].append(c["GRBM_GUI_ACTIVE"] / max(c["GRBM_COUNT"], 1))
out = {n: {k: round(statistics.median(v), 4) for k, v in a.items()} | {"launches": len(a["us"])}
       for n, a in agg.items() if len(a["us"]) >= 3}
print(json.dumps(out, indent=1))
