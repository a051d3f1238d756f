"""List where autograd will sum gradients with a PyTorch add (a tensor read by more than one autograd node): walks
the backward graph of one training loss and counts the edges that land on the same (node, input) slot."""
import collections
import sys
from pathlib import Path

import torch

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "yolo-ad-refine_amd"))
sys.path.insert(0, str(ROOT / "oracle"))
from adrefine.data.synthetic import train_batch  # noqa: E402
from adrefine.nn.tasks import DetectionModel  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else str(ROOT / "tests" / "configs" / "yolo11-701-YOLO-AD-Refine.yaml")
m = DetectionModel(cfg, compute_dtype=torch.bfloat16).cuda().train()
batch, lab = train_batch(2, 320, seed=0, device="cuda", u8=True)
b = {"img": batch["img"], **lab}
loss, _ = m(b)
hits = collections.Counter()
seen = set()
stack = [loss.grad_fn]
while stack:
    fn = stack.pop()
    if fn is None or fn in seen:
        continue
    seen.add(fn)
    for nxt, idx in fn.next_functions:
        if nxt is None:
            continue
        hits[(nxt, idx)] += 1
        stack.append(nxt)
multi = [(k, v) for k, v in hits.items() if v > 1 and type(k[0]).__name__ != "AccumulateGrad"]
by = collections.Counter()
for (fn, idx), v in multi:
    by[(type(fn).__name__, fn.name())] += v - 1
print(f"{len(multi)} slots receive more than one gradient ({sum(v - 1 for _, v in multi)} extra adds per step)")
for (t, name), n in by.most_common():
    print(f"{n:4d}  {t}  {name}")
