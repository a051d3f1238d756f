"""Probe: hipGraph capture of fork/join work on a second stream (torch.cuda.graph), pure torch, then with the
trainer at a small size. usage: python scripts/side_capture_probe.py (GPU)"""
import faulthandler
import os
import sys
import time
from pathlib import Path

faulthandler.enable()
ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "yolo-ad-refine_amd"))
import torch

dev = torch.device("cuda", 0)
side = torch.cuda.Stream(dev)
a = torch.randn(1 << 20, device=dev)
b = torch.zeros_like(a)
c = torch.zeros_like(a)


def body():
    main = torch.cuda.current_stream()
    side.wait_stream(main)
    with torch.cuda.stream(side):
        t = a * 2
        b.copy_(t)
    c.copy_(a + 1)
    main.wait_stream(side)


body()
torch.cuda.synchronize()
g = torch.cuda.CUDAGraph()
with torch.cuda.graph(g):
    body()
g.replay()
torch.cuda.synchronize()
print("pure torch fork/join capture ok", float(b.sum() - 2 * a.sum()), flush=True)

# same, no allocation on the side stream
def body2():
    main = torch.cuda.current_stream()
    side.wait_stream(main)
    with torch.cuda.stream(side):
        b.mul_(0.5)
    c.add_(1)
    main.wait_stream(side)


g2 = torch.cuda.CUDAGraph()
with torch.cuda.graph(g2):
    body2()
g2.replay()
torch.cuda.synchronize()
print("no-alloc fork/join capture ok", flush=True)

from adrefine.engine.trainer import FusedTrainer
from adrefine.data.synthetic import train_batch
from adrefine.nn.tasks import DetectionModel

model = DetectionModel(str(ROOT / "tests/configs/yolo11-701-YOLO-AD-Refine.yaml"), compute_dtype=torch.bfloat16).to(dev)
tr = FusedTrainer(model, batch_size=int(os.environ.get("BS", 8)))
batch, _ = train_batch(int(os.environ.get("BS", 8)), 320, seed=0, device=dev)
for _ in range(2):
    tr.step(batch)
torch.cuda.synchronize()
print("eager steps ok", flush=True)
tr.capture(batch)
print("capture ok", flush=True)
for _ in range(3):
    tr.step(batch)
torch.cuda.synchronize()
print("replay ok", flush=True)
