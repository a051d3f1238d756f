"""PyTorch-native device ops inside one eager bs64 bf16 train step, with the Python stack that issued each
(torch.profiler with_stack): which copies / fills / adds remain and where they come from.
usage: python scripts/torch_ops_stack.py   (GPU)"""
import sys
from collections import Counter
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "yolo-ad-refine_amd"))

import torch  # noqa: E402
from torch.profiler import ProfilerActivity, profile  # noqa: E402

from adrefine.data.synthetic import train_batch  # noqa: E402
from adrefine.engine.trainer import FusedTrainer  # noqa: E402
from adrefine.nn.tasks import DetectionModel  # noqa: E402

dev = torch.device("cuda", 0)
model = DetectionModel(str(ROOT / "tests/configs/yolo11-701-YOLO-AD-Refine.yaml"), compute_dtype=torch.bfloat16).to(dev)
tr = FusedTrainer(model, batch_size=64)
batch, _ = train_batch(64, 640, seed=0, device=dev)
for _ in range(2):
    tr.step(batch)
torch.cuda.synchronize()
WATCH = ("aten::copy_", "aten::fill_", "aten::zero_", "aten::add", "aten::add_", "aten::cat", "aten::sum",
         "aten::mul", "aten::div", "aten::clamp_min")
with profile(activities=[ProfilerActivity.CPU], with_stack=True, record_shapes=True) as prof:
    tr.step(batch)
    torch.cuda.synchronize()
cnt = Counter()
for ev in prof.events():
    if ev.name not in WATCH:
        continue
    stack = [s for s in (ev.stack or []) if "adrefine" in s or "site-packages/torch/autograd" in s][:4]
    key = (ev.name, str(ev.input_shapes)[:120], " <- ".join(s.split("/")[-1] for s in stack) or "(autograd engine)")
    cnt[key] += 1
for (name, shapes, where), n in cnt.most_common(60):
    print(f"{n:3d} {name:16s} {shapes:60s} {where}")
