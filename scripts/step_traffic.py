"""Whole-step HBM traffic of the replayed training step: per-launch PMC bytes (profiles/pmc_traffic.json, two
rocprofv3 --pmc passes over an eager bench run with the same launch mix) x each kernel's launches per replayed step
(a rocprofv3 --kernel-trace CSV of a graph-replayed bench run, steps cut at the optimizer kernel as in
replay_breakdown.py). Each kernel is normalised by ITS OWN execution count, so warm-up / capture launches and the
eager timing repeats do not leak into the per-step figure.

Calibration (MI355X_MICROARCH.md HBM section): read = 2 x FETCH_SIZE x 1 KiB holds for 16-byte-per-lane streaming
reads; other widths are uncalibrated, so the script also prints PMC read bytes / algorithmic read bytes for the
calibration kernels named in CAL (known compulsory reads, different access widths).

usage: python scripts/step_traffic.py <kernel_trace.csv> <pmc_traffic.json> <out.json> [--bs 64] [--steps 8]"""
import argparse
import csv
import json
from collections import defaultdict

ap = argparse.ArgumentParser()
ap.add_argument("trace")
ap.add_argument("pmc")
ap.add_argument("out")
ap.add_argument("--bs", type=int, default=64)
ap.add_argument("--steps", type=int, default=8)
ap.add_argument("--alg-bytes-per-img", type=float, default=210e6)
a = ap.parse_args()

rows = sorted(csv.DictReader(open(a.trace)), key=lambda r: int(r["Start_Timestamp"]))
marks = [i for i, r in enumerate(rows) if "sgd_ema" in r["Kernel_Name"]]
if len(marks) < 3:
    marks = [i for i, r in enumerate(rows) if "loss_cls_grad_kernel" in r["Kernel_Name"]]
segs = list(zip(marks[:-1], marks[1:]))[-a.steps:]
k = len(segs)
cnt, tim = defaultdict(int), defaultdict(float)
for s, e in segs:
    for r in rows[s + 1:e + 1]:
        n = r["Kernel_Name"]
        cnt[n] += 1
        tim[n] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
pmc = json.load(open(a.pmc))["kernels"]
per, missing = {}, {}
for n, c in cnt.items():
    lps = c / k
    rec = pmc.get(n)
    if rec is None:
        missing[n] = {"launches_per_step": round(lps, 2), "ms_per_step": round(tim[n] / k, 4)}
        continue
    per[n] = {"launches_per_step": round(lps, 2), "hbm_bytes_per_launch": rec["hbm_bytes_per_launch"],
              "read_bytes_per_launch": rec["read_bytes_per_launch"], "write_bytes_per_launch": rec["write_bytes_per_launch"],
              "bytes_per_step": round(lps * rec["hbm_bytes_per_launch"]), "ms_per_step": round(tim[n] / k, 4)}
tot_ms = sum(tim.values()) / k
cov_ms = sum(v["ms_per_step"] for v in per.values())
step_bytes = sum(v["bytes_per_step"] for v in per.values())
doc = {"source": f"{a.trace} ({k} replayed steps) x {a.pmc}",
       "method": "sum over kernels of PMC hbm bytes per launch x launches per replayed step; read = 2 x FETCH_SIZE "
                 "KiB (gfx950 wide-load correction), write = WRITE_SIZE KiB; Infinity-Cache hits included",
       "bs": a.bs, "steps_used": k, "kernel_ms_per_step": round(tot_ms, 3),
       "covered_ms_per_step": round(cov_ms, 3), "coverage": round(cov_ms / tot_ms, 4),
       "traffic_bytes_per_step": step_bytes, "traffic_bytes_per_img": round(step_bytes / a.bs),
       "alg_bytes_per_img": a.alg_bytes_per_img, "traffic_over_alg": round(step_bytes / a.bs / a.alg_bytes_per_img, 3),
       "traffic_gbs_over_kernel_time": round(step_bytes / (tot_ms * 1e-3) / 1e9, 1),
       "top": dict(sorted(per.items(), key=lambda kv: -kv[1]["bytes_per_step"])[:40]),
       "missing": dict(sorted(missing.items(), key=lambda kv: -kv[1]["ms_per_step"]))}
json.dump(doc, open(a.out, "w"), indent=1)
print(f"{k} steps: {step_bytes / 1e9:.2f} GB/step = {step_bytes / a.bs / 1e6:.0f} MB/img "
      f"({doc['traffic_over_alg']}x the {a.alg_bytes_per_img / 1e6:.0f} MB/img algorithmic budget), coverage "
      f"{doc['coverage']:.1%} of {tot_ms:.2f} ms kernel time; {len(missing)} kernels without PMC entries")
