"""Per-step summary of a rocprofv3 kernel_stats.csv: python scripts/kstat_summary.py <csv> <steps> [top]"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
steps = float(sys.argv[2])
top = int(sys.argv[3]) if len(sys.argv) > 3 else 40
tot = sum(float(r["TotalDurationNs"]) for r in rows) / steps / 1e6
n = sum(int(r["Calls"]) for r in rows) / steps
print(f"kernel time per step {tot:.3f} ms, launches per step {n:.1f}")
for r in rows[:top]:
    print(f"{float(r['TotalDurationNs']) / steps / 1e6:7.3f} ms {int(r['Calls']) / steps:6.1f}x "
          f"{float(r['AverageNs']) / 1e3:8.1f}us  {r['Name'][:100]}")
