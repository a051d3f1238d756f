"""Which parameters' fp32 gradients differ between the level-packed AYHead and the per-level loop after one
trainer forward_backward (tests/test_gpu_packed_head.py::test_trainer_packed_matches_levels, arena check).
usage: python scripts/packed_arena_diff.py   (GPU)"""
import sys
from pathlib import Path
ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "yolo-ad-refine_amd"))
sys.path.insert(0, str(ROOT / "tests"))
sys.path.insert(0, str(ROOT / "oracle"))  # the recipe weights the test loads (test-side only)
import torch
from adrefine.nn.tasks import DetectionModel
from adrefine.engine.trainer import FusedTrainer
from adrefine.data.synthetic import train_batch
from gpu_util import load_recipe_into

CFG = ROOT / "tests" / "configs" / "yolo11-701-YOLO-AD-Refine.yaml"


def run(packed):
    m = DetectionModel(str(CFG), compute_dtype=torch.float32)
    load_recipe_into(m)
    m = m.cuda()
    m.model[-1].packed = packed
    tr = FusedTrainer(m, batch_size=4, nbs=4)
    b0, _ = train_batch(4, 320, seed=3, device="cuda", u8=True)
    tr.forward_backward(b0)
    torch.cuda.synchronize()
    return {n: p._adr_grad.clone() for n, p in m.named_parameters() if getattr(p, "_adr_grad", None) is not None}


g0, g1 = run(False), run(True)
tot = sum(float(v.norm()) ** 2 for v in g0.values()) ** 0.5
rows = []
for n in g0:
    d = float((g1[n] - g0[n]).norm())
    rows.append((d / tot, d / max(float(g0[n].norm()), 1e-30), n))
rows.sort(reverse=True)
print(f"arena rel diff {sum(r[0] ** 2 for r in rows) ** 0.5:.3e}")
for share, rel, n in rows[:25]:
    print(f"{share:.3e} of arena  rel {rel:.3e}  {n}")
if "--all" in sys.argv:
    for n in g0:
        d = float((g1[n] - g0[n]).norm())
        print(f"rel {d / max(float(g0[n].norm()), 1e-30):.2e}  |g| {float(g0[n].norm()):.3e}  {n}")
