"""Summarise rocprofv3 kernel_stats.csv files: top kernels by total time, per-launch average (us)."""
import csv
import sys

for path in sys.argv[1:]:
    rows = list(csv.DictReader(open(path)))
    tot = sum(float(r["TotalDurationNs"]) for r in rows)
    print(f"== {path}  total {tot / 1e6:.2f} ms")
    for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:18]:
        print(f"  {r['Name'][:78]:78s} {r['Calls']:>5} {float(r['AverageNs']) / 1e3:8.1f} us {float(r['TotalDurationNs']) / tot * 100:5.1f}%")
