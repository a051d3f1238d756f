"""Training checkpoints in the reference's layout (engine/trainer.py:507-540 save_model, :718-744 resume_training).

The reference pickles `{'epoch', 'best_fitness', 'model': None, 'ema': <whole EMA nn.Module, half>, 'updates',
'optimizer': <SGD state_dict, fp16 buffers>, 'train_args', 'train_metrics', 'train_results', 'date', 'version',
'license', 'docs'}`. This build writes the same keys with the same meaning, with one deliberate difference:
'ema' holds the EMA's state_dict (the reference's 541 key names and shapes, fp16) instead of a pickled module, so
a checkpoint loads with `torch.load(..., weights_only=True)` — nothing in the file executes. 'optimizer' is a
torch.optim.SGD state_dict laid out exactly as the reference's build_optimizer creates it (param_groups in the
order g2 biases, g0 decayed weights, g1 norm weights — trainer.py:798-808 — parameters numbered in that order,
momentum buffers fp16 like utils/torch_utils.convert_optimizer_state_dict_to_fp16), so
`torch.optim.SGD(...).load_state_dict(ckpt['optimizer'])` accepts it on the reference side.

Resume follows resume_training: the model AND the EMA start from ckpt['ema'] (the reference resumes the model
from the EMA weights of last.pt), momentum buffers from ckpt['optimizer'], EMA update count from
ckpt['updates'], start_epoch = epoch + 1.
"""
from __future__ import annotations

import io
from datetime import datetime
from pathlib import Path

import torch

VERSION = "adrefine-8.3.9"  # the reference's ultralytics version string is 8.3.9 (ultralytics/__init__.py:3)


def _ref_param_order(trainer):
    """(name, group) of every trainable parameter in the reference optimizer's numbering: g2, then g0, then g1."""
    by_group = {0: [], 1: [], 2: []}
    for name, _p, grp, isp in trainer.entries:
        if isp:
            by_group[grp].append(name)
    # entries are stage-major; the reference numbers parameters in named_modules order within each group
    order = {n: i for i, (n, _) in enumerate(trainer.model.named_parameters())}
    for g in by_group.values():
        g.sort(key=lambda n: order[n])
    return [(n, 2) for n in by_group[2]] + [(n, 0) for n in by_group[0]] + [(n, 1) for n in by_group[1]]


def optimizer_state_dict(trainer):
    """torch.optim.SGD state_dict of the trainer's momentum buffers, reference grouping, fp16 buffers."""
    idx = {name: i for i, (name, _p, _g, isp) in enumerate(trainer.entries) if isp}
    state, groups = {}, {2: [], 0: [], 1: []}
    for k, (name, grp) in enumerate(_ref_param_order(trainer)):
        ei = idx[name]
        _, t, _, _ = trainer.entries[ei]
        if trainer.updates > 0 and getattr(t, "_adr_used", False):
            off = trainer._goff[ei]
            state[k] = {"momentum_buffer": trainer.mom[off:off + t.numel()].view(t.shape).detach().half().cpu()}
        groups[grp].append(k)
    lrs = {0: trainer.lr[0], 1: trainer.lr[1], 2: trainer.lr[2]}
    wds = {0: trainer.wd, 1: 0.0, 2: 0.0}
    pg = [{"lr": lrs[g], "momentum": trainer.momentum, "dampening": 0, "weight_decay": wds[g], "nesterov": True,
           "maximize": False, "foreach": None, "differentiable": False, "fused": None,
           "initial_lr": trainer.sched.lr0, "params": groups[g]} for g in (2, 0, 1)]
    return {"state": state, "param_groups": pg}


def ema_state_dict_half(trainer):
    """The EMA model's full state_dict in the model's key order: floating entries from the EMA (fp16, as the
    reference's .half()), integer buffers (BN num_batches_tracked) as the EMA copy holds them — the value at trainer
    construction, since ModelEMA.update skips non-floating entries (utils/torch_utils.py:536-541)."""
    ema = trainer.ema_state_dict()
    out = {}
    for k, v in trainer.model.state_dict().items():
        if v.dtype.is_floating_point:
            out[k] = ema[k].detach().half().cpu().clone()
        else:
            out[k] = trainer.ema_int.get(k, v).detach().cpu().clone()
    return out


def save_checkpoint(trainer, path, epoch, best_fitness=None, train_args=None, train_metrics=None,
                    train_results=None):
    """save_model (trainer.py:507-540): one serialised buffer written to `path`."""
    buf = io.BytesIO()
    torch.save({
        "epoch": int(epoch),
        "best_fitness": best_fitness,
        "model": None,  # resume and final checkpoints derive from EMA
        "ema": ema_state_dict_half(trainer),
        "updates": int(trainer.updates),
        "optimizer": optimizer_state_dict(trainer),
        "train_args": dict(train_args or {}),
        "train_metrics": dict(train_metrics or {}),
        "train_results": dict(train_results or {}),
        "date": datetime.now().isoformat(),
        "version": VERSION,
        "license": "AGPL-3.0 (https://ultralytics.com/license)",
        "docs": "https://docs.ultralytics.com",
    }, buf)
    Path(path).write_bytes(buf.getvalue())


def load_checkpoint(path):
    """torch.load with weights_only=True (nothing in the file executes)."""
    return torch.load(path, map_location="cpu", weights_only=True)


def resume(trainer, ckpt):
    """resume_training (trainer.py:718-744) into a FusedTrainer built on the same model: returns
    (start_epoch, best_fitness)."""
    start_epoch = ckpt.get("epoch", -1) + 1
    assert start_epoch > 0, "checkpoint marks training as finished"
    ema = {k: (v.float() if v.is_floating_point() else v) for k, v in ckpt["ema"].items()}
    # the model resumes from the EMA weights (reference: attempt_load_weights(last) loads ckpt['ema'])
    trainer.model.load_state_dict({k: v.to(trainer.dev) for k, v in ema.items()}, strict=True)
    for ei, (name, t, _, _) in enumerate(trainer.entries):
        off = trainer._eoff[ei]
        trainer.ema_flat[off:off + t.numel()].copy_(ema[name].reshape(-1).to(trainer.dev))
    best_fitness = 0.0
    opt = ckpt.get("optimizer")
    if opt is not None:
        order = _ref_param_order(trainer)
        idx = {name: i for i, (name, _p, _g, isp) in enumerate(trainer.entries) if isp}
        for k, (name, _grp) in enumerate(order):
            st = opt["state"].get(k) or opt["state"].get(str(k))
            if st is None:
                continue
            ei = idx[name]
            t = trainer.entries[ei][1]
            off = trainer._goff[ei]
            trainer.mom[off:off + t.numel()].copy_(st["momentum_buffer"].float().reshape(-1).to(trainer.dev))
        best_fitness = ckpt.get("best_fitness") or 0.0
    trainer.updates = int(ckpt.get("updates", 0))
    trainer.packs.valid = False
    # the batch counter restarts at the resumed epoch (ni = i + nb * epoch: trainer.py:370); _do_train resets
    # last_opt_step to -1 (trainer.py:331), so the first batch after a resume always runs the optimizer
    trainer.ni = start_epoch * trainer.sched.nb if trainer.sched.nb else 0
    trainer.last_opt_step = -1
    return start_epoch, best_fitness
