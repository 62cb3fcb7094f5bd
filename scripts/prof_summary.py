"""Summarise a rocprofv3 kernel_stats.csv: share of time, calls, average per kernel (per step if --steps)."""
import csv
import sys

path = sys.argv[1]
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 1
rows = list(csv.DictReader(open(path)))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
print(f"total {tot / 1e6:.2f} ms  ({tot / 1e6 / steps:.3f} ms/step over {steps})")
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[: int(sys.argv[3]) if len(sys.argv) > 3 else 40]:
    print(f"{float(r['TotalDurationNs']) / tot * 100:5.1f}% {float(r['TotalDurationNs']) / 1e3 / steps:8.1f}us/step "
          f"calls={r['Calls']:>5} avg={float(r['AverageNs']) / 1e3:8.1f}us  {r['Name'][:140]}")
