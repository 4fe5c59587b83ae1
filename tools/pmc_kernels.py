"""Per-kernel-name summary of three rocprofv3 --pmc passes (FETCH_SIZE, WRITE_SIZE, TCC_HIT/MISS):
mean bytes per launch (FETCH doubled per the gfx950 note) and L2 hit rate.
usage: python tools/pmc_kernels.py <fetch_dir> <write_dir> <l2_dir>"""
import collections
import csv
import json
import sys
from pathlib import Path


def load(d):
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for r in csv.DictReader(open(Path(d) / "run_counter_collection.csv")):
        name = r["Kernel_Name"].split("(")[0][:90]
        agg[name][r["Counter_Name"]].append(float(r["Counter_Value"]))
    return agg


f, w, l2 = (load(d) for d in sys.argv[1:4])
out = {}
for name in f:
    fe = f[name].get("FETCH_SIZE", [0])
    wr = w.get(name, {}).get("WRITE_SIZE", [0])
    hit = sum(l2.get(name, {}).get("TCC_HIT_sum", [0]))
    miss = sum(l2.get(name, {}).get("TCC_MISS_sum", [0]))
    out[name] = {"launches": len(fe), "fetch_bytes": 2 * 1024 * sum(fe) / len(fe),
                 "write_bytes": 1024 * sum(wr) / max(len(wr), 1), "l2_hit_rate": hit / max(hit + miss, 1)}
print(json.dumps(out, indent=1))
