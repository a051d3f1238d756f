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


_CACHE = {}


def _ours(dtype):
    if dtype not in _CACHE:
        _CACHE[dtype] = _train(dtype)
    return _CACHE[dtype]


def test_bf16_trains_like_fp32():
    l32, u32, n32 = _ours(torch.float32)
    l16, u16, n16 = _ours(torch.bfloat16)
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


def test_bf16_gap_vs_reference_fp16_amp():
    """the reference trains with fp16 autocast + GradScaler (engine/trainer.py:269, 383, 393), so
    its own arithmetic already moves the trajectory away from fp32. The oracle (tests/bf16_sim.oracle_train) runs
    the same 50 steps on the device in fp32 and under fp16 autocast; the bf16 HIP trajectory's gap to the fp32 HIP
    trajectory (per-step relative gap of the total loss) is bounded by 1.5x the fp16-AMP gap over the same steps,
    in mean and in max.

    The AMP run is taken with the GradScaler already settled (init_scale = the scale the reference's default 2^16
    start reaches after the same 50 steps, here 16): from 2^16 the loss (x batch size) overflows fp16 in the
    backward, so the first ~13 steps are skipped, and that trajectory lags fp32 by up to 434x at step 14 before it
    catches up (printed below, not bounded). Measured (round 5): bf16 HIP vs fp32 HIP mean 0.031, max 0.107;
    fp16-AMP (settled) vs fp32 oracle mean 0.060, max 0.175 — ratios 0.52 / 0.61; fp32 HIP vs fp32 oracle itself
    drifts to mean 0.023, max 0.095 over the 50 steps (the trajectory amplifies last-bit differences)."""
    import time

    from bf16_sim import oracle_train
    from adrefine.data.synthetic import labels
    from adrefine.engine.trainer import param_groups
    from adrefine.nn.tasks import DetectionModel
    from recipe import recipe_state_dict
    from conftest import state_dict_spec
    l32, _, _ = _ours(torch.float32)
    l16, _, _ = _ours(torch.bfloat16)
    groups = [[n for n, _ in g] for g in param_groups(DetectionModel(str(CFG)))]
    P = recipe_state_dict([(k, s) for k, s, _ in state_dict_spec("701")])
    from adrefine.data.synthetic import images_u8
    x = images_u8(BS, S, seed=21).float() / 255.0
    lab = labels(BS, 80, seed=22)
    t0 = time.time()
    o32, _ = oracle_train(P, CFG, groups, x, lab, STEPS, amp_fp16=False)
    o16, scale = oracle_train(P, CFG, groups, x, lab, STEPS, amp_fp16=True)
    o16c, _ = oracle_train(P, CFG, groups, x, lab, STEPS, amp_fp16=True, init_scale=scale)
    gap = lambda a, b: ((a.sum(1) - b.sum(1)).abs() / b.sum(1).abs())  # noqa: E731
    g_ours, g_amp, g_ampc, g_anchor = gap(l16, l32), gap(o16, o32), gap(o16c, o32), gap(o32, l32)
    print(f"oracle runs {time.time() - t0:.1f}s; settled GradScaler scale {scale}")
    for name, g in (("fp32 HIP vs fp32 oracle", g_anchor), ("bf16 HIP vs fp32 HIP", g_ours),
                    ("fp16-AMP (scaler from 2^16) vs fp32 oracle", g_amp),
                    ("fp16-AMP (settled scaler) vs fp32 oracle", g_ampc)):
        print(f"{name}: max {float(g.max()):.4f} mean {float(g.mean()):.4f} last-10 max {float(g[-10:].max()):.4f}")
    print("per-step", [round(float(a), 4) for a in g_ours], [round(float(a), 4) for a in g_ampc])
    assert float(g_ours.mean()) <= 1.5 * float(g_ampc.mean()), (float(g_ours.mean()), float(g_ampc.mean()))
    assert float(g_ours.max()) <= 1.5 * float(g_ampc.max()), (float(g_ours.max()), float(g_ampc.max()))
