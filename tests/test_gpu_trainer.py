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
    tr = FusedTrainer(m, lr0=0.01, momentum=0.937, weight_decay=5e-4, nbs=2, batch_size=2)  # accumulate 1
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
    wd = 5e-4 * 2 * max(round(2 / 2), 1) / 2
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


def _oracle_model():
    P = recipe_state_dict([(k, s) for k, s, _ in state_dict_spec("701")])
    d = yaml.safe_load(CFG.read_text())
    layers, save = O.parse(d, 3, None)
    for k, v in P.items():
        if v.dtype.is_floating_point and "running" not in k and not k.endswith("dfl.conv.weight"):
            v.requires_grad_(True)
    return P, layers, save


def _oracle_opt(P, groups, used, wd, lr=0.01, momentum=0.937):
    opt = torch.optim.SGD([P[k] for k in groups[2] if k in used], lr=lr, momentum=momentum, nesterov=True)
    opt.add_param_group({"params": [P[k] for k in groups[0] if k in used], "weight_decay": wd})
    opt.add_param_group({"params": [P[k] for k in groups[1] if k in used], "weight_decay": 0.0})
    return opt


def _worst_update(sd, P, used):
    worst = 0.0
    for k in used:
        a, b = sd[k].detach().cpu(), P[k].detach()
        delta = (b - recipe_state_dict([(k, b.shape)])[k]).abs().max()
        worst = max(worst, float((a - b).abs().max()) / (float(delta) + 1e-12))
    return worst


def test_accumulate_steps_every_4_batches():
    """batch 2 with nbs 8 -> accumulate 4 (trainer.py:305): four fwd+bwd passes sum into the gradient arena and
    only the 4th batch runs clip + SGD + EMA + zero_grad (trainer.py:396-398, 580-588)."""
    from adrefine.engine.trainer import FusedTrainer, param_groups
    from adrefine.nn.tasks import DetectionModel
    m = DetectionModel(str(CFG))
    load_recipe_into(m)
    groups = [[n for n, _ in g] for g in param_groups(m)]
    m = m.cuda()
    tr = FusedTrainer(m, lr0=0.01, momentum=0.937, weight_decay=5e-4, nbs=8, batch_size=2)
    assert tr.accumulate == 4
    w0 = m.state_dict()["model.0.conv.weight"].clone()
    batches = [(synthetic_images(2, 320, seed=10 + i), synthetic_labels(2, 80, seed=20 + i)) for i in range(4)]
    for i, (x, lab) in enumerate(batches):
        tr.step({"img": x.cuda(), **lab})
        torch.cuda.synchronize()
        if i < 3:
            assert tr.updates == 0 and torch.equal(m.state_dict()["model.0.conv.weight"], w0)
            assert float(tr.grad.abs().max()) > 0  # gradients accumulating, not zeroed
    assert tr.updates == 1 and tr.last_opt_step == 3
    assert float(tr.grad.abs().max()) == 0.0  # zero_grad after the step
    P, layers, save = _oracle_model()
    for x, lab in batches:
        preds = O.forward(P, layers, save, x, train=True)
        loss, _ = O.detection_loss(preds, lab["batch_idx"], lab["cls"], lab["bboxes"])
        loss.backward()  # accumulates in .grad
    used = [k for k in P if P[k].requires_grad and P[k].grad is not None]
    opt = _oracle_opt(P, groups, used, wd=5e-4 * 2 * 4 / 8)
    tn = torch.nn.utils.clip_grad_norm_([P[k] for k in used], max_norm=10.0)
    assert abs(float(tr.norm) - float(tn)) <= 1e-3 * float(tn), (float(tr.norm), float(tn))
    opt.step()
    worst = _worst_update(m.state_dict(), P, used)
    assert worst < 2e-2, worst


def test_warmup_lr_momentum_two_steps():
    """Warm-up (trainer.py:369-381, nb 10 -> nw 100): step 0 runs with bias lr 0.1, weight lr 0, momentum 0.8;
    step 1 with the interpolated values — two trainer steps vs the oracle + torch SGD with those groups."""
    from adrefine.engine.trainer import FusedTrainer, Schedule, param_groups
    from adrefine.nn.tasks import DetectionModel
    m = DetectionModel(str(CFG))
    load_recipe_into(m)
    groups = [[n for n, _ in g] for g in param_groups(m)]
    m = m.cuda()
    tr = FusedTrainer(m, nbs=2, batch_size=2, nb=10, epochs=100)
    sch = Schedule(nbs=2, batch_size=2, nb=10, epochs=100)
    batches = [(synthetic_images(2, 320, seed=30 + i), synthetic_labels(2, 80, seed=40 + i)) for i in range(2)]
    P, layers, save = _oracle_model()
    used = None
    opt = None
    for ni, (x, lab) in enumerate(batches):
        tr.step({"img": x.cuda(), **lab})
        lrs, mom, acc = sch.at(ni)
        assert acc == 1 and tr.lr == lrs and tr.momentum == mom
        preds = O.forward(P, layers, save, x, train=True)
        loss, _ = O.detection_loss(preds, lab["batch_idx"], lab["cls"], lab["bboxes"])
        loss.backward()
        if opt is None:
            used = [k for k in P if P[k].requires_grad and P[k].grad is not None]
            opt = _oracle_opt(P, groups, used, wd=5e-4)
        for pg, lr in zip(opt.param_groups, (lrs[2], lrs[0], lrs[1])):  # (g2, g0, g1) order
            pg["lr"], pg["momentum"] = lr, mom
        torch.nn.utils.clip_grad_norm_([P[k] for k in used], max_norm=10.0)
        opt.step()
        opt.zero_grad()
    assert tr.updates == 2
    worst = _worst_update(m.state_dict(), P, used)
    assert worst < 3e-2, worst
