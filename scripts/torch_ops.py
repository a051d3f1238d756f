"""Which PyTorch-native ops still run inside the train step (copies, fills, adds): one eager bs64 step under
torch.profiler (CPU ops only); every aten copy/fill/add event is attributed to its outermost autograd node or
Python-level parent op. usage: python scripts/torch_ops.py   (GPU)"""
import sys
from collections import Counter
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "yolo-ad-refine_amd"))

import torch
from torch.profiler import ProfilerActivity, profile

from adrefine.data.synthetic import train_batch
from adrefine.engine.trainer import FusedTrainer
from adrefine.nn.tasks import DetectionModel

dev = torch.device("cuda", 0)
model = DetectionModel(str(ROOT / "tests/configs/yolo11-701-YOLO-AD-Refine.yaml"), compute_dtype=torch.bfloat16).to(dev)
tr = FusedTrainer(model, batch_size=64)
batch, _ = train_batch(64, 640, seed=0, device=dev)
for _ in range(2):
    tr.step(batch)
torch.cuda.synchronize()

WATCH = ("aten::copy_", "aten::fill_", "aten::zero_", "aten::add", "aten::add_", "aten::to", "aten::clone",
         "aten::contiguous", "aten::zeros", "aten::zeros_like", "aten::cat", "aten::sum", "aten::mul")
with profile(activities=[ProfilerActivity.CPU], with_stack=False) as prof:
    tr.step(batch)
    torch.cuda.synchronize()

cnt = Counter()
for ev in prof.events():
    if ev.name not in WATCH:
        continue
    chain = []
    p = ev.cpu_parent
    while p is not None:
        chain.append(p.name)
        p = p.cpu_parent
    # nearest autograd node / Python op, then the outermost frame
    near = next((c for c in chain if "autograd" in c or "Backward" in c or not c.startswith("aten::")), "(top)")
    cnt[(ev.name, near[:90], chain[0][:40] if chain else "")] += 1
for (name, near, par), n in cnt.most_common(70):
    print(f"{n:4d}  {name:16s} {par:40s} {near}")
