"""Evidence that the benchmarked bf16 path TRAINS like the parity-pinned fp32 path: 50
optimizer steps of SGD-nesterov + clip + EMA (engine/trainer.py:383-398, optimizer_step :580-588) from the recipe
weights on one fixed batch (701-n, 320^2, bs 8, 8 COCO-shape labels per image on average), once in the fp32 parity
mode (elementwise within 1e-4 of the reference oracle for one step, tests/test_gpu_trainer.py) and once in bf16
(the bench's dtype), both through captured hipGraphs.

Bounds (stated; set from the measured run with margin — fp32 8037 -> 6.74, bf16 8169 -> 7.28 over the 50 steps,
per-step total-loss gap 0.6-11 % (largest late, where the loss is 1000x smaller), final items box / cls / dfl
28 % / 3 % / 11 % apart, update-vector cosine 0.867, norm difference 0.3 %):
* both runs train: the total loss falls below 1 % of its first value;
* loss trajectory: per-step relative gap at most 20 %, mean over the 50 steps at most 6 %, final total within 15 %;
* parameters: the bf16 total update vector (final - initial, all trainable parameters) has cosine >= 0.8 with the
  fp32 one and relative norm difference <= 5 %.
The gap is what bf16 storage (8-bit significand) does through batch-statistics BatchNorm (the ideal-bf16
restatement of the oracle already differs from fp32 by 17-33 % relative L2 in the train-mode head outputs); the
reference trains with fp16 autocast instead."""
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
    print(f"mean rel gap {float(rel.mean()):.4f}")
    assert t32[-1] <= 0.01 * t32[0] and t16[-1] <= 0.01 * t16[0], (t32, t16)
    assert float(rel.max()) <= 0.20 and float(rel.mean()) <= 0.06 and float(rel[-1]) <= 0.15, rel
    assert cos >= 0.8 and dn <= 0.05, (cos, dn)
