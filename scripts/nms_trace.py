"""Median adr_nms kernel duration per nms_micro.py setting from a rocprofv3 kernel trace (dev tool).
usage: python scripts/nms_trace.py <kernel_trace.csv> [per_setting_calls=53] [warmup=3]"""
import csv
import statistics
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
per = int(sys.argv[2]) if len(sys.argv) > 2 else 53
warm = int(sys.argv[3]) if len(sys.argv) > 3 else 3
names = ["predict", "val", "synth_predict", "synth_val"]
k = [r for r in rows if "nms" in r["Kernel_Name"]]
kinds = sorted({r["Kernel_Name"] for r in k})
calls_per = max(1, len(k) // (per * len(names)))  # kernels per NMS call (1 persistent, 6 chain)
d = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in k]
tot = [sum(d[i:i + calls_per]) for i in range(0, len(d), calls_per)]
out = {}
for i, n in enumerate(names):
    seg = tot[i * per + warm:(i + 1) * per]
    if seg:
        out[n] = round(statistics.median(seg), 1)
print(kinds if len(kinds) > 1 else kinds[0][:40], out)
