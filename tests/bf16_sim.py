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
