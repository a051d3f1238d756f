"""Mona adapter — HIP-backed drop-ins for the reference's ultralytics/nn/modules/mona.py (used by the 697 L10
variant). Same class names, constructor signatures and parameter names, so state_dicts load unchanged."""
from __future__ import annotations

import torch
import torch.nn as nn

from ... import kernels as K


class LayerNorm2d(nn.LayerNorm):
    """LayerNorm over the channels of each pixel (mona.py:5-10)."""

    def forward(self, x):
        C = x.shape[1]
        one = torch.ones(C, device=x.device)
        return K.ln_mix(x, self.weight, self.bias, one, torch.zeros(C, device=x.device), self.eps)


class MonaOp(nn.Module):
    """mona.py:12-33: (dw3 + dw5 + dw7) / 3 + x, then + 1x1 projector."""

    def __init__(self, in_features):
        super().__init__()
        self.conv1 = nn.Conv2d(in_features, in_features, kernel_size=3, padding=3 // 2, groups=in_features)
        self.conv2 = nn.Conv2d(in_features, in_features, kernel_size=5, padding=5 // 2, groups=in_features)
        self.conv3 = nn.Conv2d(in_features, in_features, kernel_size=7, padding=7 // 2, groups=in_features)
        self.projector = nn.Conv2d(in_features, in_features, kernel_size=1)
        self.register_buffer("_third", torch.full((3,), 1.0 / 3.0), persistent=False)

    def forward(self, x):
        ys = [K.dwconv(x, c.weight, c.bias, k) for c, k in ((self.conv1, 3), (self.conv2, 5), (self.conv3, 7))]
        t = K.weighted_sum(self._third, ys, base=x)
        p, _ = K.conv2d(t, self.projector.weight, self.projector.bias, 1, 0)
        return K.add(t, p)


class Mona(nn.Module):
    """mona.py:35-65: x + project2(dropout(gelu(MonaOp(project1(LN(x) * gamma + x * gammax)))))."""

    def __init__(self, in_dim):
        super().__init__()
        self.project1 = nn.Conv2d(in_dim, 64, 1)
        self.project2 = nn.Conv2d(64, in_dim, 1)
        self.dropout = nn.Dropout(p=0.1)
        self.adapter_conv = MonaOp(64)
        self.norm = LayerNorm2d(in_dim)
        self.gamma = nn.Parameter(torch.ones(in_dim, 1, 1) * 1e-6)
        self.gammax = nn.Parameter(torch.ones(in_dim, 1, 1))
        # device seed of the dropout mask stream (advanced on the device after every use)
        self.register_buffer("_seed", torch.randint(0, 2 ** 62, (1,), dtype=torch.int64), persistent=False)

    def forward(self, x, hw_shapes=None):
        z = K.ln_mix(x, self.norm.weight, self.norm.bias, self.gamma, self.gammax, self.norm.eps)
        p1, _ = K.conv2d(z, self.project1.weight, self.project1.bias, 1, 0)
        a = K.act(self.adapter_conv(p1), "gelu")
        a = K.dropout(a, self.dropout.p, self._seed, self.training)
        p2, _ = K.conv2d(a, self.project2.weight, self.project2.bias, 1, 0)
        return K.add(x, p2)
