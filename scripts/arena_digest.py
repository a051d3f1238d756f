"""Gradient arena + loss items of one fp32 trainer forward_backward (bs 4, 320^2, recipe weights) saved to a file,
for bitwise A/B of two library builds (ADR_LIB); usage: python scripts/arena_digest.py OUT.pt [--compare A.pt B.pt]"""
import sys
from pathlib import Path
ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "yolo-ad-refine_amd"))
sys.path.insert(0, str(ROOT / "tests"))
sys.path.insert(0, str(ROOT / "oracle"))  # the recipe weights the tests load (test-side only)
import torch
if sys.argv[1] == "--compare":
    a, b = torch.load(sys.argv[2]), torch.load(sys.argv[3])
    for k in a:
        print(k, "bitwise" if torch.equal(a[k], b[k]) else f"DIFF max {float((a[k] - b[k]).abs().max()):.3e}")
    sys.exit(0)
from adrefine.nn.tasks import DetectionModel
from adrefine.engine.trainer import FusedTrainer
from adrefine.data.synthetic import train_batch
from gpu_util import load_recipe_into
m = DetectionModel(str(ROOT / "tests/configs/yolo11-701-YOLO-AD-Refine.yaml"), compute_dtype=torch.float32)
load_recipe_into(m)
m = m.cuda()
tr = FusedTrainer(m, batch_size=4, nbs=4)
b0, _ = train_batch(4, 320, seed=3, device="cuda", u8=True)
items = tr.forward_backward(b0)
torch.cuda.synchronize()
torch.save({"arena": tr.grad.detach().cpu(), "items": torch.as_tensor(items).float().cpu()}, sys.argv[1])
print("saved", sys.argv[1])
