"""Where the step's HIP runtime copies (__amd_rocclr_copyBuffer: hipMemcpyAsync device-to-device) and fills come
from: one eager bf16 train step (701-n, 640^2, bs 64) under torch.profiler with Python stacks; prints the aten ops
that launched device copies / fills, grouped by their innermost adrefine frame. usage: python scripts/copy_sites.py"""
import collections
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "yolo-ad-refine_amd"))
import torch  # noqa: E402
from torch.profiler import ProfilerActivity, profile  # noqa: E402

from adrefine.data.synthetic import train_batch  # noqa: E402
from adrefine.engine.trainer import FusedTrainer  # noqa: E402
from adrefine.nn.tasks import DetectionModel  # noqa: E402

dev = torch.device("cuda", 0)
torch.manual_seed(0)
m = DetectionModel(str(ROOT / "tests/configs/yolo11-701-YOLO-AD-Refine.yaml"), compute_dtype=torch.bfloat16).to(dev)
tr = FusedTrainer(m, batch_size=64)
batch, _ = train_batch(64, 640, seed=0, device=dev, u8=True)
for _ in range(2):
    tr.step(batch)
torch.cuda.synchronize()
with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], with_stack=True) as prof:
    tr.step(batch)
    torch.cuda.synchronize()
sites = collections.Counter()
for ev in prof.events():
    if ev.name not in ("aten::copy_", "aten::clone", "aten::contiguous", "aten::fill_", "aten::zero_", "aten::cat",
                       "aten::to", "aten::_to_copy", "aten::index_put_", "aten::zeros", "aten::ones", "aten::full"):
        continue
    stack = [f for f in (ev.stack or []) if "adrefine" in f or "bench" in f or "trainer" in f]
    where = stack[0] if stack else "(no adrefine frame)"
    sites[(ev.name, where)] += 1
for (name, where), n in sites.most_common(40):
    print(f"{n:4d}  {name:18s} {where}")
kinds = collections.Counter(e.name for e in prof.events() if e.device_type == torch.autograd.DeviceType.CUDA)
print({k: v for k, v in kinds.items() if "copy" in k.lower() or "fill" in k.lower() or "memset" in k.lower()})
