"""Where the elementwise launches of one eager train step come from: every adr_ew launch labelled with its op,
size and call site (kernels.timing_detail), aggregated per call site. usage: python scripts/ew_sites.py [--scale n --img 640 --bs 64] (GPU)"""
import argparse
import sys
from collections import defaultdict
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "yolo-ad-refine_amd"))
import torch

import adrefine.kernels as K
from adrefine.data.synthetic import train_batch
from adrefine.engine.trainer import FusedTrainer
from adrefine.nn.tasks import DetectionModel

ap = argparse.ArgumentParser()
ap.add_argument("--scale", default="n")
ap.add_argument("--img", type=int, default=640)
ap.add_argument("--bs", type=int, default=64)
args = ap.parse_args()
dev = torch.device("cuda", 0)
cfg = ROOT / "tests/configs/yolo11-701-YOLO-AD-Refine.yaml"
if args.scale != "n":
    import yaml
    d = yaml.safe_load(open(cfg))
    d["scale"] = args.scale
    model = DetectionModel(d, compute_dtype=torch.bfloat16).to(dev)
else:
    model = DetectionModel(str(cfg), compute_dtype=torch.bfloat16).to(dev)
tr = FusedTrainer(model, batch_size=args.bs)
batch, _ = train_batch(args.bs, args.img, seed=0, device=dev)
for _ in range(2):
    tr.step(batch)
torch.cuda.synchronize()
K.TIMING_REPEAT = 1
K.FANOUT_LOG = []
K.timing_begin()
tr.step(batch)
K.timing_end()
fan = defaultdict(int)
for rec in K.FANOUT_LOG:
    fan[rec] += 1
print("fan-out backward: (site, autograd grads, sink buf, seeded slice, pending adds, shape) x count")
for rec, n in sorted(fan.items(), key=lambda kv: str(kv[0])):
    if rec[1] + int(rec[2]) + rec[4] >= 2:  # something left to sum here
        print(f"  {n:3d}x {rec}")
agg = defaultdict(lambda: [0, 0.0, 0])
for tag, shape, nb, fl, t in K.timing_detail():
    if "ew_kernel" not in tag:
        continue
    op, _, rest = shape.partition(" ")
    site = rest.split("@")[-1]
    a = agg[(site, op)]
    a[0] += 1
    a[1] += t
    a[2] += nb or 0
tot = sum(v[1] for v in agg.values())
print(f"adr_ew: {sum(v[0] for v in agg.values())} launches, {1e3 * tot:.2f} ms (eager, events)")
for (site, op), (n, t, nb) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
    print(f"{1e3 * t:7.3f} ms {n:4d}x  {op:8s} {site}  ({nb / max(t, 1e-12) / 1e9:.0f} GB/s)")
