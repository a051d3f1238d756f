"""An 'ideal bf16' restatement of the reference for the bf16 parity bounds: the CPU oracle (fp32 arithmetic)
with the output of every torch.nn.functional op it calls rounded to bfloat16, and the gradient flowing back
into it likewise — i.e. bf16 storage of every intermediate and of every activation gradient, nothing else. Its distance to the fp32 fixtures is the divergence that bf16 storage alone
causes on this network; tests/test_gpu_bf16.py requires the HIP bf16 path to stay within a stated factor of
it. (Test infrastructure: imports the oracle.)"""
import types

import torch
import torch.nn.functional as Freal
import yaml

import adr_oracle as O


class _Round(torch.autograd.Function):
    """bf16 storage of a value in the forward and of its gradient in the backward."""

    @staticmethod
    def forward(ctx, t):
        return t.bfloat16().float()

    @staticmethod
    def backward(ctx, g):
        return g.bfloat16().float()


def _rnd(t):
    if torch.is_tensor(t) and t.is_floating_point():
        return _Round.apply(t)
    if isinstance(t, (tuple, list)):
        return type(t)(_rnd(u) for u in t)
    return t


class _Bf16F(types.ModuleType):
    def __getattr__(self, n):
        f = getattr(Freal, n)
        if callable(f):
            return lambda *a, **k: _rnd(f(*a, **k))
        return f


def oracle_forward(P, cfg, x, train, bf16):
    """O.forward on the parsed yaml (a path or an already-loaded dict), with bf16 rounding of every functional
    op's output when bf16."""
    d = cfg if isinstance(cfg, dict) else yaml.safe_load(open(cfg).read())
    layers, save = O.parse(d, 3, None)
    prev = O.F
    O.F = _Bf16F("F") if bf16 else Freal
    try:
        return O.forward(P, layers, save, _rnd(x) if bf16 else x, train=train)
    finally:
        O.F = prev


def oracle_train(P, cfg, groups, x, lab, steps, amp_fp16, lr=0.01, momentum=0.937, wd=5e-4, device="cuda",
                 init_scale=2.0 ** 16):
    """`steps` optimizer steps of the oracle network on one batch with the reference's training arithmetic:
    amp_fp16=True runs each forward + loss under torch.autocast(float16) with a GradScaler, as the reference trains
    (engine/trainer.py:269 scaler, :383 autocast, :393 scaler.scale(loss).backward(), optimizer_step :580-588:
    unscale_, clip_grad_norm_(10), scaler.step, update); amp_fp16=False is the same loop in fp32. SGD nesterov with
    the trainer's three parameter groups (`groups`: [decay weights, BN weights, biases] names). Runs on `device`
    (factory calls inside the oracle are redirected there). init_scale: the GradScaler's starting scale (the
    reference's default 2^16; a calibrated value skips the scaler's first overflow-and-halve steps). Returns
    ((steps, 3) loss items, final scale). (Test infrastructure: drives the oracle; nothing here is on the product
    path.)"""
    d = cfg if isinstance(cfg, dict) else yaml.safe_load(open(cfg).read())
    layers, save = O.parse(d, 3, None)
    P = {k: v.detach().to(device).clone() for k, v in P.items()}
    for k, v in P.items():
        if v.dtype.is_floating_point and "running" not in k and not k.endswith("dfl.conv.weight"):
            v.requires_grad_(True)
    x = x.to(device)
    lab = {k: v.to(device) for k, v in lab.items()}
    scaler = torch.amp.GradScaler("cuda", init_scale=init_scale, enabled=amp_fp16)
    opt, used, out = None, None, []
    prev = torch.get_default_device()
    torch.set_default_device(device)
    try:
        for _ in range(steps):
            with torch.autocast("cuda", dtype=torch.float16, enabled=amp_fp16):
                preds = O.forward(P, layers, save, x, train=True)
                loss, items = O.detection_loss(preds, lab["batch_idx"], lab["cls"], lab["bboxes"])
            scaler.scale(loss).backward()
            if opt is None:
                used = [k for k in P if P[k].requires_grad and P[k].grad is not None]
                opt = torch.optim.SGD([P[k] for k in groups[2] if k in used], lr=lr, momentum=momentum, nesterov=True)
                opt.add_param_group({"params": [P[k] for k in groups[0] if k in used], "weight_decay": wd})
                opt.add_param_group({"params": [P[k] for k in groups[1] if k in used], "weight_decay": 0.0})
            scaler.unscale_(opt)
            torch.nn.utils.clip_grad_norm_([P[k] for k in used], max_norm=10.0)
            scaler.step(opt)
            scaler.update()
            opt.zero_grad()
            out.append(items.detach().float().cpu())
    finally:
        torch.set_default_device(prev)
    return torch.stack(out).double(), float(scaler.get_scale()) if amp_fp16 else 1.0
