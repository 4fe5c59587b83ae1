"""Per-configuration kernel durations from the rocprofv3 kernel trace of tools/es_kernel_probe.py:
dispatches in start order, (2 + 6 * iters) per configuration (noise + fitness warm-up, then per
iteration noise, perturb, fitness, update (caps off), update + caps).  Prints median µs per kernel.
usage: python tools/es_prof_summary.py <kernel_trace.csv> [iters]"""
import csv
import statistics
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
it = int(sys.argv[2]) if len(sys.argv) > 2 else 20
rows = [r for r in rows if "eggroll" in r["Kernel_Name"]]
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
per = 2 + 6 * it
names = ["rank 1 pop 8", "rank 1 pop 64", "rank 1 pop 128", "rank 4 pop 128"]
for c, name in enumerate(names):
    seg = rows[c * per:(c + 1) * per][2:]
    d = {}
    for i, r in enumerate(seg):
        slot = ["noise", "perturb", "fitness", "update(no caps)", "update(caps)", "caps"][i % 6]
        d.setdefault(slot, []).append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    print(name, {k: round(statistics.median(v), 2) for k, v in d.items()})
