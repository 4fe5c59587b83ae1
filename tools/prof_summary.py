"""Summarise a rocprofv3 --stats kernel CSV (diagnostic)."""
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
print(f"total kernel time {tot / 1e9:.3f} s")
for r in rows[: int(sys.argv[2]) if len(sys.argv) > 2 else 40]:
    print(f"{float(r['TotalDurationNs']) / 1e9:8.3f}s {float(r['Percentage']):6.2f}% n={r['Calls']:>6} "
          f"avg={float(r['AverageNs']) / 1e3:10.1f}us  {r['Name'][:120]}")
