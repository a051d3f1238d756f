"""Print the top kernels of a rocprofv3 kernel_stats.csv per step. usage: python scripts/kstats.py <csv> <steps> [filter...]"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
steps = float(sys.argv[2])
flt = sys.argv[3:]
tot = sum(float(r["TotalDurationNs"]) for r in rows)
print(f"total kernel time per step: {tot / steps / 1e6:.3f} ms")
for r in rows:
    n = r["Name"]
    if flt and not any(f in n for f in flt):
        continue
    print(f"{float(r['TotalDurationNs']) / steps / 1e3:9.1f} us/step {int(r['Calls']) / steps:7.1f}/step "
          f"{float(r['AverageNs']) / 1e3:8.2f} us  {n[:100]}")
