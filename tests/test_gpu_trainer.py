"""GPU parity: one full training step (fwd + loss + bwd + clip_grad_norm_(10) + SGD nesterov with the
reference's 3 parameter groups + EMA) vs the CPU oracle driven through torch.optim.SGD (trainer.py:580-588)."""
import math

import pytest
import torch
import yaml

import adr_oracle as O
from conftest import ROOT, state_dict_spec
from gpu_util import assert_close, load_recipe_into
from recipe import recipe_state_dict, synthetic_images, synthetic_labels

pytestmark = pytest.mark.gpu
CFG = ROOT / "tests" / "configs" / "yolo11-701-YOLO-AD-Refine.yaml"


def test_train_step_matches_oracle_sgd():
    from adrefine.engine.trainer import FusedTrainer, param_groups
    from adrefine.nn.tasks import DetectionModel
    m = DetectionModel(str(CFG))
    load_recipe_into(m)
    groups = [[n for n, _ in g] for g in param_groups(m)]
    m = m.cuda()
    tr = FusedTrainer(m, lr0=0.01, momentum=0.937, weight_decay=5e-4, batch_size=2)
    x = synthetic_images(2, 320, seed=0)
    lab = synthetic_labels(2, 80, seed=1)
    items = tr.step({"img": x.cuda(), **lab})
    # oracle: same step on CPU
    P = recipe_state_dict([(k, s) for k, s, _ in state_dict_spec("701")])
    d = yaml.safe_load(CFG.read_text())
    layers, save = O.parse(d, 3, None)
    for k, v in P.items():
        if v.dtype.is_floating_point and "running" not in k and not k.endswith("dfl.conv.weight"):
            v.requires_grad_(True)
    preds = O.forward(P, layers, save, x, train=True)
    loss, ritems = O.detection_loss(preds, lab["batch_idx"], lab["cls"], lab["bboxes"])
    assert_close(items, ritems, rtol=1e-4, atol=1e-5, what="loss items")
    loss.backward()
    used = [k for k in P if P[k].requires_grad and P[k].grad is not None]
    wd = 5e-4 * 2 * max(round(64 / 2), 1) / 64
    opt = torch.optim.SGD([P[k] for k in groups[2] if k in used], lr=0.01, momentum=0.937, nesterov=True)
    opt.add_param_group({"params": [P[k] for k in groups[0] if k in used], "weight_decay": wd})
    opt.add_param_group({"params": [P[k] for k in groups[1] if k in used], "weight_decay": 0.0})
    tn = torch.nn.utils.clip_grad_norm_([P[k] for k in used], max_norm=10.0)
    assert abs(float(tr.norm) - float(tn)) <= 1e-3 * float(tn)
    opt.step()
    sd = m.state_dict()
    worst = 0.0
    for k in used:
        a, b = sd[k].detach().cpu(), P[k].detach()
        delta = (b - recipe_state_dict([(k, b.shape)])[k]).abs().max()  # size of the update itself
        err = float((a - b).abs().max())
        worst = max(worst, err / (float(delta) + 1e-12))
    assert worst < 2e-2, worst  # the update step matches to ~1% of its own magnitude
    # EMA: d = 0.9999 * (1 - exp(-1/2000)) after the first update
    dd = 0.9999 * (1 - math.exp(-1 / 2000))
    ema = tr.ema_state_dict()
    k = "model.0.conv.weight"
    init = recipe_state_dict([(k, P[k].shape)])[k]
    assert_close(ema[k].cpu(), dd * init + (1 - dd) * sd[k].cpu(), rtol=1e-5, atol=1e-6, what="ema")
