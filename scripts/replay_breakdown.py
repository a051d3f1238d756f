"""Per-step GPU time of the REPLAYED training steps only, from a rocprofv3 --kernel-trace CSV of a bench.py run:
steps are cut at the once-per-step optimizer kernel (sgd_ema; the loss kernel when the optimizer steps less often), the last `--steps` complete ones are averaged (the
eager warm-up / capture steps, which launch differently, are left out). Prints the family table (families of
kernel_breakdown.py), the top kernels and the launch count per step.
With --pmc profiles/pmc_traffic.json every kernel row also carries its measured HBM bytes per launch (PMC passes of
the same launch mix), the bandwidth they amount to over the kernel's replayed average duration, and that bandwidth
as a fraction of the 8 TB/s HBM peak (`hbm frac`: the roofline position of what the kernel actually moves).
usage: python scripts/replay_breakdown.py <run_kernel_trace.csv> [--steps 8] [--top 40] [--pmc pmc_traffic.json]"""
import argparse
import csv
import sys
from collections import defaultdict
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent))
from kernel_breakdown import FAMILIES  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("trace")
ap.add_argument("--steps", type=int, default=8)
ap.add_argument("--top", type=int, default=40)
ap.add_argument("--pmc", default=None)
a = ap.parse_args()
rows = sorted(csv.DictReader(open(a.trace)), key=lambda r: int(r["Start_Timestamp"]))
marks = [i for i, r in enumerate(rows) if "sgd_ema" in r["Kernel_Name"]]
if len(marks) < 3:  # gradient accumulation (bs < nbs: the optimizer runs every few steps): cut at the loss kernel
    marks = [i for i, r in enumerate(rows) if "loss_cls_grad_kernel" in r["Kernel_Name"]]
segs = list(zip(marks[:-1], marks[1:]))[-a.steps:]
fam = defaultdict(lambda: [0.0, 0])
ker = defaultdict(lambda: [0.0, 0])
span = 0.0
for s, e in segs:
    span += (int(rows[e]["End_Timestamp"]) - int(rows[s]["End_Timestamp"])) / 1e6
    for r in rows[s + 1:e + 1]:
        n = r["Kernel_Name"]
        t = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
        f = next((f for f, keys in FAMILIES if any(k in n for k in keys)), "other")
        fam[f][0] += t
        fam[f][1] += 1
        ker[n][0] += t
        ker[n][1] += 1
k = len(segs)
tot = sum(v[0] for v in fam.values()) / k
print(f"{k} replayed steps: {sum(v[1] for v in fam.values()) / k:.0f} launches, kernel time {tot:.2f} ms, "
      f"wall {span / k:.2f} ms per step")
print("| family | ms / step | launches / step | share |\n|---|---|---|---|")
for f, (ms, n) in sorted(fam.items(), key=lambda kv: -kv[1][0]):
    print(f"| {f} | {ms / k:.2f} | {n / k:.0f} | {100 * ms / k / tot:.1f} % |")
import json  # noqa: E402
pmc = json.load(open(a.pmc))["kernels"] if a.pmc else {}
if pmc:
    print(f"\n| kernel | ms / step | launches / step | avg us | PMC MB / launch | TB/s | hbm frac |\n"
          f"|---|---|---|---|---|---|---|")
else:
    print(f"\n| kernel | ms / step | launches / step | avg us |\n|---|---|---|---|")
for n, (ms, c) in sorted(ker.items(), key=lambda kv: -kv[1][0])[:a.top]:
    row = f"| {n[:110]} | {ms / k:.3f} | {c / k:.0f} | {1e3 * ms / c:.1f} |"
    if pmc:
        rec = pmc.get(n)
        if rec is None:
            row += " – | – | – |"
        else:
            tbs = rec["hbm_bytes_per_launch"] / (ms / c * 1e-3) / 1e12
            row += f" {rec['hbm_bytes_per_launch'] / 1e6:.1f} | {tbs:.2f} | {tbs / 8.0:.3f} |"
    print(row)
