"""Per-conv-shape timing table of one eager train step (HIP events around every conv GEMM launch).
usage: python scripts/conv_table.py [--bs 64] [--steps 2] [--scale l --img 1280] [--top N]   (GPU)"""
import argparse
import sys
from collections import defaultdict
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "yolo-ad-refine_amd"))

ap = argparse.ArgumentParser()
ap.add_argument("--bs", type=int, default=64)
ap.add_argument("--steps", type=int, default=2)
ap.add_argument("--scale", default="n")
ap.add_argument("--img", type=int, default=640)
ap.add_argument("--top", type=int, default=200)
ap.add_argument("--by-gap", action="store_true", help="sort by time above the attainable roofline (8 TB/s, 2.5 PF)")
args = ap.parse_args()

import torch
import adrefine.kernels as K
from adrefine.engine.trainer import FusedTrainer
from adrefine.data.synthetic import train_batch
from adrefine.nn.tasks import DetectionModel

dev = torch.device("cuda", 0)
import yaml
cfg = yaml.safe_load((ROOT / "tests/configs/yolo11-701-YOLO-AD-Refine.yaml").read_text())
cfg["scale"] = args.scale
torch.manual_seed(0)
model = DetectionModel(cfg, compute_dtype=torch.bfloat16).to(dev)
tr = FusedTrainer(model, batch_size=args.bs)
batch, _ = train_batch(args.bs, args.img, seed=0, device=dev, u8=True)
for _ in range(2):
    tr.step(batch)
torch.cuda.synchronize()
K.timing_begin()
for _ in range(args.steps):
    tr.step(batch)
K.timing_end()
agg = defaultdict(lambda: [0, 0, 0.0, 0.0])
for tag, shape, nb, fl, t in K.timing_detail():  # every timed libadr launch, keyed by kernel + shape
    a = agg[f"{tag[:48]:48s} {shape}"]
    a[0] += 1; a[1] += nb or 0; a[2] += fl or 0; a[3] += t
tot = sum(v[3] for v in agg.values()) / args.steps
print(f"timed total per step: {1e3 * tot:.2f} ms")
def att(v):  # attainable time of the entry's launches: max(bytes / HBM peak, flops / bf16 MFMA peak) per launch
    n, nb, fl, t = v
    return n * max(nb / n / 8e12, fl / n / 2.5e15)


key = (lambda kv: -(kv[1][3] - att(kv[1]))) if args.by_gap else (lambda kv: -kv[1][3])
for shape, (n, nb, fl, t) in sorted(agg.items(), key=key)[:args.top]:
    a = att((n, nb, fl, t))
    print(f"{1e3 * t / args.steps:7.3f} ms {n // args.steps:3d}x {1e6 * t / n:8.1f}us {nb / t / 1e9:7.0f} GB/s "
          f"{fl / t / 1e12:6.1f} TF/s  att {a / t:5.2f} gap {1e3 * (t - a) / args.steps:6.3f} ms  {shape}")
