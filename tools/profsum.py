"""Summarise a rocprofv3 --stats kernel_stats.csv (per translate call)."""
import csv
import sys

path = sys.argv[1]
calls = float(sys.argv[2]) if len(sys.argv) > 2 else 1.0
rows = list(csv.DictReader(open(path)))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:25]:
    print(f"{float(r['TotalDurationNs'])/1e6/calls:9.3f} ms/call {float(r['Percentage']):6.2f}% n={int(r['Calls'])/calls:8.1f} "
          f"avg={float(r['AverageNs'])/1e3:9.2f}us  {r['Name'][:100]}")
print(f"total {tot/1e6/calls:.3f} ms/call")
