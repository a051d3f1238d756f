"""Summarise a rocprofv3 kernel_stats.csv per step: python scripts/prof_summary.py <csv> <steps> [top]"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
steps = float(sys.argv[2])
top = int(sys.argv[3]) if len(sys.argv) > 3 else 40
tot = sum(float(r["TotalDurationNs"]) for r in rows)
calls = sum(int(r["Calls"]) for r in rows)
print(f"total {tot / steps / 1e6:.2f} ms/step, {calls / steps:.0f} launches/step")
for r in rows[:top]:
    print(f"{float(r['TotalDurationNs']) / steps / 1e6:7.3f} ms {int(r['Calls']) / steps:6.1f}x {float(r['AverageNs']) / 1e3:8.1f}us  "
          f"{r['Name'][:100]}")
