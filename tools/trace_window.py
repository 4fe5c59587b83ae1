"""Per-kernel stats of a rocprofv3 kernel trace restricted to the bench's timed region.

bench.py launches eggroll's k_philox_words once right before and once right after the timed
epochs (markers); this script keeps only dispatches strictly between the first two markers.
usage: python tools/trace_window.py gpurun_out/<dir>/run_kernel_trace.csv [top] [--json out.json]
"""
import csv, json, sys
from collections import defaultdict

path = sys.argv[1]
top = int(sys.argv[2]) if len(sys.argv) > 2 and not sys.argv[2].startswith("--") else 40
rows = list(csv.DictReader(open(path)))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
marks = [i for i, r in enumerate(rows) if "k_philox_words" in r["Kernel_Name"]]
if len(marks) >= 2:
    lo, hi = marks[0] + 1, marks[1]
else:
    lo, hi = 0, len(rows)
win = rows[lo:hi]
t0, t1 = int(win[0]["Start_Timestamp"]), int(win[-1]["End_Timestamp"])
agg = defaultdict(lambda: [0, 0.0])
for r in win:
    d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    a = agg[r["Kernel_Name"]]
    a[0] += 1
    a[1] += d
tot = sum(v[1] for v in agg.values())
print(f"window: {len(win)} dispatches, wall {(t1 - t0) / 1e9:.3f} s, kernel-busy {tot / 1e6:.3f} s (markers: {len(marks)})")
items = sorted(agg.items(), key=lambda kv: -kv[1][1])
for name, (n, us) in items[:top]:
    print(f"{us / 1e6:8.3f}s {100 * us / tot:6.2f}% n={n:>6} avg={us / n:10.1f}us  {name[:110]}")
if "--json" in sys.argv:
    out = sys.argv[sys.argv.index("--json") + 1]
    json.dump({"window_wall_s": (t1 - t0) / 1e9, "kernel_busy_s": tot / 1e6,
               "kernels": [{"name": k, "calls": n, "total_us": us, "avg_us": us / n} for k, (n, us) in items]},
              open(out, "w"), indent=1)
