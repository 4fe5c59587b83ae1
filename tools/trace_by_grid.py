"""Summarise a rocprofv3 kernel-trace CSV by (kernel, grid size): launches, mean / median duration (us).
Kernels of one name launched at several shapes (a probe sweeping shapes) are told apart by their grid.
usage: python tools/trace_by_grid.py <kernel_trace.csv> [name-substring ...]"""
import csv
import statistics
import sys
from collections import defaultdict


def main(path, subs):
    rows = defaultdict(list)
    with open(path, newline="") as f:
        for r in csv.DictReader(f):
            name = r["Kernel_Name"]
            if subs and not any(s in name for s in subs):
                continue
            grid = r.get("Grid_Size_X") or r.get("Grid_Size") or "?"
            rows[(name[:90], grid)].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    for (name, grid), d in sorted(rows.items(), key=lambda kv: -sum(kv[1])):
        print(f"{name:90s} grid={grid:>10s} n={len(d):4d} mean={statistics.mean(d):9.1f} "
              f"median={statistics.median(d):9.1f} us")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2:])
