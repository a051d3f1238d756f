"""(P, C) of every BatchNorm finalize launch of one eager 701-n train step (bs 64, 640^2): P = partial rows the
finalize reduces per channel. usage: python scripts/finalize_sites.py (GPU)"""
import sys
from collections import Counter
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "yolo-ad-refine_amd"))
import torch
import adrefine.native as native
from adrefine.data.synthetic import train_batch
from adrefine.engine.trainer import FusedTrainer
from adrefine.nn.tasks import DetectionModel

dev = torch.device("cuda", 0)
model = DetectionModel(str(ROOT / "tests/configs/yolo11-701-YOLO-AD-Refine.yaml"), compute_dtype=torch.bfloat16).to(dev)
tr = FusedTrainer(model, batch_size=64)
batch, _ = train_batch(64, 640, seed=0, device=dev, u8=True)
tr.step(batch)
torch.cuda.synchronize()
seen = Counter()


def hook(name, fn, a):
    if name in ("adr_bn_finalize", "adr_bn_bwd_finalize") and a[0] is not None:
        seen[(name, int(a[1]), int(a[2]))] += 1
    return fn(*a)


native.CALL_HOOK = hook
tr.step(batch)
torch.cuda.synchronize()
native.CALL_HOOK = None
tot = Counter()
for (n, P, C), k in sorted(seen.items(), key=lambda kv: (kv[0][0], -kv[0][1])):
    print(f"{n:22s} P {P:6d} C {C:4d}  x{k}")
    tot[n] += k
print(dict(tot))
