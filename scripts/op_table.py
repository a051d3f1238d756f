"""Per-entry-point timing table of one eager train step: every libadr_hip call bracketed by HIP events
(adrefine.native.OP_TRACE), grouped by (entry point, caller, integer arguments). Torch-side kernels are not
covered (they show up in rocprofv3 only).
usage: python scripts/op_table.py [--bs 64] [--steps 1] [--top 80]   (GPU)"""
import argparse
import sys
from collections import defaultdict
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "yolo-ad-refine_amd"))

ap = argparse.ArgumentParser()
ap.add_argument("--bs", type=int, default=64)
ap.add_argument("--steps", type=int, default=1)
ap.add_argument("--top", type=int, default=80)
args = ap.parse_args()

import torch
import adrefine.native as NV
from adrefine.engine.trainer import FusedTrainer
from adrefine.data.synthetic import train_batch
from adrefine.nn.tasks import DetectionModel

dev = torch.device("cuda", 0)
model = DetectionModel(str(ROOT / "tests/configs/yolo11-701-YOLO-AD-Refine.yaml"), compute_dtype=torch.bfloat16).to(dev)
tr = FusedTrainer(model, batch_size=args.bs)
batch, _ = train_batch(args.bs, 640, seed=0, device=dev)
for _ in range(2):
    tr.step(batch)
torch.cuda.synchronize()
NV.OP_TRACE = []
for _ in range(args.steps):
    tr.step(batch)
torch.cuda.synchronize()
recs, NV.OP_TRACE = NV.OP_TRACE, None
by_site = defaultdict(lambda: [0, 0.0])
by_name = defaultdict(lambda: [0, 0.0])
for name, caller, ints, e0, e1 in recs:
    t = e0.elapsed_time(e1) * 1e-3
    a = by_site[(name, caller, ints)]
    a[0] += 1
    a[1] += t
    b = by_name[name]
    b[0] += 1
    b[1] += t
tot = sum(v[1] for v in by_name.values()) / args.steps
print(f"traced libadr time per step: {1e3 * tot:.2f} ms over {len(recs) // args.steps} calls")
print("--- by entry point ---")
for name, (n, t) in sorted(by_name.items(), key=lambda kv: -kv[1][1]):
    print(f"{1e3 * t / args.steps:7.3f} ms {n // args.steps:4d}x {1e6 * t / n:8.1f}us  {name}")
print("--- by call site ---")
for (name, caller, ints), (n, t) in sorted(by_site.items(), key=lambda kv: -kv[1][1])[:args.top]:
    print(f"{1e3 * t / args.steps:7.3f} ms {n // args.steps:3d}x {1e6 * t / n:8.1f}us  {name} [{caller}] {ints}")
