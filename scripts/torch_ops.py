"""Which PyTorch-native ops still run inside the train step (copies, fills, adds): one eager bs64 step under
torch.profiler with Python stacks, aggregated by (op, innermost adrefine frame).
usage: python scripts/torch_ops.py   (GPU)"""
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
with profile(activities=[ProfilerActivity.CPU], with_stack=True) as prof:
    tr.step(batch)
    torch.cuda.synchronize()
cnt = Counter()
for ev in prof.events():
    if ev.name not in ("aten::copy_", "aten::fill_", "aten::add", "aten::add_", "aten::zero_", "aten::clone",
                       "aten::contiguous", "aten::cat", "aten::mul", "aten::sum", "aten::to", "aten::_to_copy"):
        continue
    frames = [f for f in (ev.stack or []) if "adrefine" in f or "torch/autograd" in f]
    site = frames[0] if frames else "(no adrefine frame)"
    cnt[(ev.name, site)] += 1
for (name, site), n in cnt.most_common(60):
    print(f"{n:4d}  {name:18s} {site}")
