"""Checkpoint layout (engine/checkpoint.py) vs the reference's save_model / resume_training
(engine/trainer.py:507-540, 718-744): same keys, EMA + fp16, the optimizer state_dict a reference-grouped
torch.optim.SGD accepts, and a resume that restores model (from the EMA), EMA, momentum and update count.
CPU only: the trainer's host-side tables and buffers are built without running a step."""
import torch

from conftest import ROOT
from gpu_util import load_recipe_into

CFG = ROOT / "tests" / "configs" / "yolo11-701-YOLO-AD-Refine.yaml"
KEYS = {"epoch", "best_fitness", "model", "ema", "updates", "optimizer", "train_args", "train_metrics",
        "train_results", "date", "version", "license", "docs"}


def _trainer(seed):
    from adrefine.engine.trainer import FusedTrainer
    from adrefine.nn.tasks import DetectionModel
    m = DetectionModel(str(CFG))
    load_recipe_into(m)
    g = torch.Generator().manual_seed(seed)
    with torch.no_grad():
        for p in m.parameters():
            p.add_(0.01 * torch.randn(p.shape, generator=g))
    tr = FusedTrainer(m, batch_size=16, nb=100, epochs=10)
    return tr, g


def test_save_load_resume(tmp_path):
    from adrefine.engine import checkpoint as C
    from adrefine.engine.trainer import param_groups
    tr, g = _trainer(1)
    for _, t, _, isp in tr.entries:
        if isp:
            t._adr_used = True
    tr.mom.copy_(torch.randn(tr.mom.shape, generator=g))
    tr.ema_flat.add_(0.05 * torch.randn(tr.ema_flat.shape, generator=g))
    tr.updates = 37
    f = tmp_path / "last.pt"
    C.save_checkpoint(tr, f, epoch=4, best_fitness=0.3, train_args={"batch": 16}, train_metrics={"fitness": 0.3})
    ck = C.load_checkpoint(f)
    assert set(ck) == KEYS and ck["model"] is None and ck["epoch"] == 4 and ck["updates"] == 37
    sd = tr.model.state_dict()
    assert list(ck["ema"]) == list(sd) and len(sd) == 541
    assert all(v.dtype == torch.float16 for v in ck["ema"].values() if v.is_floating_point())
    # the reference's optimizer (build_optimizer grouping: g2, g0, g1) loads it
    groups = param_groups(tr.model)
    params = dict(tr.model.named_parameters())
    opt = torch.optim.SGD([params[n] for n, _ in groups[2]], lr=0.01, momentum=0.937, nesterov=True)
    opt.add_param_group({"params": [params[n] for n, _ in groups[0]], "weight_decay": tr.wd})
    opt.add_param_group({"params": [params[n] for n, _ in groups[1]], "weight_decay": 0.0})
    opt.load_state_dict(ck["optimizer"])
    ema = tr.ema_state_dict()
    for ei, (name, t, _, isp) in enumerate(tr.entries):
        if not isp:
            continue
        off = tr._goff[ei]
        buf = opt.state[params[name]]["momentum_buffer"]
        assert torch.equal(buf.float(), tr.mom[off:off + t.numel()].view(t.shape).half().float()), name
    # resume into a trainer on a differently initialised model
    tr2, _ = _trainer(2)
    start, best = C.resume(tr2, ck)
    assert start == 5 and best == 0.3 and tr2.updates == 37 and tr2.ni == 500 and tr2.last_opt_step == -1
    # reference (trainer.py:331, 396): the first batch after a resume steps the optimizer (accumulate is 4 here)
    assert tr2.sched.at(tr2.ni)[2] == 4 and tr2.will_step()
    sd2, ema2 = tr2.model.state_dict(), tr2.ema_state_dict()
    for k in sd:
        if not sd[k].is_floating_point():
            continue
        assert torch.equal(sd2[k], ema[k].half().float()), k
        assert torch.equal(ema2[k], ema[k].half().float()), k
    assert torch.equal(tr2.mom, tr.mom.half().float())
