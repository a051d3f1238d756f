"""Evidence that the benchmarked bf16 path TRAINS like the parity-pinned fp32 path: 50
optimizer steps of SGD-nesterov + clip + EMA (engine/trainer.py:383-398, optimizer_step :580-588) from the recipe
weights on one fixed batch (701-n, 320^2, bs 8, 8 COCO-shape labels per image on average), once in the fp32 parity
mode (elementwise within 1e-4 of the reference oracle for one step, tests/test_gpu_trainer.py) and once in bf16
(the bench's dtype), both through captured hipGraphs.

Bounds (stated; the measured values are printed and recorded in DESIGN.md §4):
* loss trajectory: at every step the bf16 total loss is within 5 % of the fp32 one, and over the last 10 steps
  within 3 %; both must fall by at least 20 % from step 0 (the run actually trains);
* per-item (box, cls, dfl) at the final step within 10 %;
* parameters: the bf16 total update vector (final - initial, all trainable parameters) has cosine >= 0.9 with the
  fp32 one and relative norm difference <= 15 %."""
import pytest
import torch

from conftest import ROOT

pytestmark = pytest.mark.gpu
CFG = ROOT / "tests" / "configs" / "yolo11-701-YOLO-AD-Refine.yaml"
STEPS, BS, S = 50, 8, 320


def _train(dtype):
    from adrefine.data.synthetic import train_batch
    from adrefine.engine.trainer import FusedTrainer
    from adrefine.nn.tasks import DetectionModel
    from gpu_util import load_recipe_into
    m = DetectionModel(str(CFG), compute_dtype=dtype)
    load_recipe_into(m)
    m = m.cuda()
    names = [n for n, p in m.named_parameters() if p.requires_grad]
    init = torch.cat([p.detach().float().reshape(-1) for _, p in m.named_parameters() if p.requires_grad]).clone()
    batch, _ = train_batch(BS, S, seed=21, device="cuda", u8=True)
    tr = FusedTrainer(m, batch_size=BS, nbs=BS)  # accumulate 1: an optimizer step per batch
    losses = [tr.step(batch).float().clone()]
    tr.capture(batch)
    for _ in range(STEPS - 1):
        losses.append(tr.step(batch).float().clone())  # (a replay returns the same static tensor)
    torch.cuda.synchronize()
    final = torch.cat([p.detach().float().reshape(-1) for _, p in m.named_parameters() if p.requires_grad])
    return torch.stack(losses).cpu().double(), (final - init).cpu().double(), names


def test_bf16_trains_like_fp32():
    l32, u32, n32 = _train(torch.float32)
    l16, u16, n16 = _train(torch.bfloat16)
    assert n32 == n16
    assert torch.isfinite(l32).all() and torch.isfinite(l16).all()
    t32, t16 = l32.sum(1), l16.sum(1)
    rel = ((t16 - t32).abs() / t32.abs())
    cos = float((u16 @ u32) / (u16.norm() * u32.norm()))
    dn = float((u16.norm() - u32.norm()).abs() / u32.norm())
    items_final = ((l16[-1] - l32[-1]).abs() / l32[-1].abs())
    print(f"fp32 loss {t32[0]:.3f} -> {t32[-1]:.3f}; bf16 {t16[0]:.3f} -> {t16[-1]:.3f}; max rel gap "
          f"{float(rel.max()):.4f} (last 10: {float(rel[-10:].max()):.4f}); final items rel "
          f"{items_final.tolist()}; update cosine {cos:.4f}, norm diff {dn:.4f}")
    assert t32[-1] <= 0.8 * t32[0] and t16[-1] <= 0.8 * t16[0], (t32, t16)
    assert float(rel.max()) <= 0.05 and float(rel[-10:].max()) <= 0.03, rel
    assert float(items_final.max()) <= 0.10, items_final
    assert cos >= 0.9 and dn <= 0.15, (cos, dn)
