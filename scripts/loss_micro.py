"""Time v8DetectionLoss forward + backward (adr_det_loss, one launch sequence) at the bench shape: bs 64, 640^2
head outputs (bf16 NHWC), synthetic COCO-shape labels; HIP events over R calls."""
import sys
from pathlib import Path

import torch

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "yolo-ad-refine_amd"))
from adrefine.data.synthetic import labels  # noqa: E402
from adrefine.nn.modules.head import AYHead  # noqa: E402
from adrefine.utils.loss import v8DetectionLoss  # noqa: E402


class _M:
    def __init__(self):
        self.model = [AYHead(80, [128, 128, 128])]
        self.args = None


bs, S, R = 64, 640, 20
g = torch.Generator().manual_seed(0)
feats = [(torch.randn(bs, 144, S // s, S // s, generator=g) * 2).to("cuda", torch.bfloat16)
         .contiguous(memory_format=torch.channels_last).requires_grad_(True) for s in (8, 16, 32)]
lab = labels(bs, 80, seed=1)
batch = {"batch_idx": lab["batch_idx"], "cls": lab["cls"], "bboxes": lab["bboxes"]}
crit = v8DetectionLoss(_M())
for _ in range(3):
    loss, items = crit(feats, batch)
    loss.backward()
torch.cuda.synchronize()
a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
a.record()
for _ in range(R):
    loss, items = crit(feats, batch)
    loss.backward()
b.record()
torch.cuda.synchronize()
print(f"loss fwd+bwd {1e3 * a.elapsed_time(b) / R:.1f} us  loss={float(loss):.6f} items={items.tolist()}")
