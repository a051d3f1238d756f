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
ap.add_argument("--top", type=int, default=150)
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


def est_bytes(name, ints):
    """Algorithmic HBM bytes of the streaming entry points (integer arguments in call order; pointers dropped;
    the trailing stream handle is dropped too)."""
    ints = ints[:-1] if ints and ints[-1] == 0 else ints
    try:
        es = 2 if ints[0] == 1 else 4
        if name == "adr_affine_act" and len(ints) == 10:
            N, HW, C = ints[7:10]
            return 2 * N * HW * C * es
        if name == "adr_affine_act_bwd" and len(ints) == 14:
            N, HW, C, acc = ints[10:14]
            return (3 + acc) * N * HW * C * es
        if name == "adr_nc_reduce" and len(ints) == 12:
            mode, (N, HW, C) = ints[1], ints[8:11]
            return (2 if mode == 1 else 1) * N * HW * C * es
        if name == "adr_ew" and len(ints) == 10:
            op, npix, C, acc = ints[1], ints[7], ints[8], ints[9]
            ops = {0: 2, 1: 3, 2: 3, 3: 4, 4: 2, 5: 3, 6: 4}[op] + acc
            return ops * npix * C * es
    except (IndexError, KeyError):
        pass
    return None
by_site = defaultdict(lambda: [0, 0.0, 0])
by_name = defaultdict(lambda: [0, 0.0])
for name, caller, ints, e0, e1 in recs:
    t = e0.elapsed_time(e1) * 1e-3
    a = by_site[(name, caller, ints)]
    a[0] += 1
    a[1] += t
    a[2] += est_bytes(name, ints) or 0
    b = by_name[name]
    b[0] += 1
    b[1] += t
tot = sum(v[1] for v in by_name.values()) / args.steps
print(f"traced libadr time per step: {1e3 * tot:.2f} ms over {len(recs) // args.steps} calls")
print("--- by entry point ---")
for name, (n, t) in sorted(by_name.items(), key=lambda kv: -kv[1][1]):
    print(f"{1e3 * t / args.steps:7.3f} ms {n // args.steps:4d}x {1e6 * t / n:8.1f}us  {name}")
print("--- by call site ---")
for (name, caller, ints), (n, t, nb) in sorted(by_site.items(), key=lambda kv: -kv[1][1])[:args.top]:
    bw = f"{nb / t / 1e9:6.0f} GB/s" if nb else "          "
    print(f"{1e3 * t / args.steps:7.3f} ms {n // args.steps:3d}x {1e6 * t / n:8.1f}us {bw}  {name} [{caller}] {ints}")
print("--- streaming entry points: achieved bandwidth by name ---")
agg = defaultdict(lambda: [0.0, 0])
for (name, caller, ints), (n, t, nb) in by_site.items():
    if nb:
        agg[name][0] += t
        agg[name][1] += nb
for name, (t, nb) in sorted(agg.items(), key=lambda kv: -kv[1][0]):
    print(f"{1e3 * t / args.steps:7.3f} ms  {nb / t / 1e9:6.0f} GB/s  {nb / args.steps / 1e6:8.1f} MB/step  {name}")
