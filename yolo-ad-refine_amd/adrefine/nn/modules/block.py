"""Backbone / neck blocks — HIP-backed drop-ins for the reference's ultralytics/nn/modules/block.py.

Same class names, constructor signatures and parameter names as the reference (so the z-yaml configs and
state_dicts load unchanged); forward passes are compositions of libadr_hip kernels on NHWC activations.
Channel splits (C2f chunk, C2PSA split) are zero-copy NHWC views; concatenations are one copy per piece.
"""
from __future__ import annotations

import math

import torch
import torch.nn as nn

from ... import kernels as K
from .conv import Conv, Conv2d

__all__ = ("Bottleneck", "C2f", "C3", "C3k", "C3k2", "SPPF", "MLCA", "Bottleneck_MLCA", "C3k_MLCA", "C3k2_MLCA",
           "ELA_HSFPN", "Multiply", "Add", "Fusion", "DFL")


class Bottleneck(nn.Module):
    """Standard bottleneck (reference block.py:341-354)."""

    def __init__(self, c1, c2, shortcut=True, g=1, k=(3, 3), e=0.5):
        super().__init__()
        c_ = int(c2 * e)
        self.cv1 = Conv(c1, c_, k[0], 1)
        self.cv2 = Conv(c_, c2, k[1], 1, g=g)
        self.add = shortcut and c1 == c2

    def forward(self, x):
        y = self.cv2(self.cv1(x))
        return K.add(x, y) if self.add else y


class C2f(nn.Module):
    """CSP bottleneck with 2 convolutions (reference block.py:232-247)."""

    def __init__(self, c1, c2, n=1, shortcut=False, g=1, e=0.5):
        super().__init__()
        self.c = int(c2 * e)
        self.cv1 = Conv(c1, 2 * self.c, 1, 1)
        self.cv2 = Conv((2 + n) * self.c, c2, 1)
        self.m = nn.ModuleList(Bottleneck(self.c, self.c, shortcut, g, k=((3, 3), (3, 3)), e=1.0) for _ in range(n))

    def forward(self, x):
        ys = list(K.split(self.cv1(x), (self.c, self.c)))  # chunk(2, 1): NHWC views, no copy
        for m in self.m:
            ys.append(m(ys[-1]))
        return self.cv2(K.cat(ys))


class C3(nn.Module):
    """CSP bottleneck with 3 convolutions (reference block.py:256-270)."""

    def __init__(self, c1, c2, n=1, shortcut=True, g=1, e=0.5):
        super().__init__()
        c_ = int(c2 * e)
        self.cv1 = Conv(c1, c_, 1, 1)
        self.cv2 = Conv(c1, c_, 1, 1)
        self.cv3 = Conv(2 * c_, c2, 1)
        self.m = nn.Sequential(*(Bottleneck(c_, c_, shortcut, g, k=((1, 1), (3, 3)), e=1.0) for _ in range(n)))

    def forward(self, x):
        return self.cv3(K.cat([self.m(self.cv1(x)), self.cv2(x)]))


class C3k(C3):
    """C3 with k x k bottlenecks (reference block.py:742-750)."""

    def __init__(self, c1, c2, n=1, shortcut=True, g=1, e=0.5, k=3):
        super().__init__(c1, c2, n, shortcut, g, e)
        c_ = int(c2 * e)
        self.m = nn.Sequential(*(Bottleneck(c_, c_, shortcut, g, k=(k, k), e=1.0) for _ in range(n)))


class C3k2(C2f):
    """C2f with C3k or Bottleneck blocks (reference block.py:731-739)."""

    def __init__(self, c1, c2, n=1, c3k=False, e=0.5, g=1, shortcut=True):
        super().__init__(c1, c2, n, shortcut, g, e)
        self.m = nn.ModuleList(
            C3k(self.c, self.c, 2, shortcut, g) if c3k else Bottleneck(self.c, self.c, shortcut, g) for _ in range(n))


class SPPF(nn.Module):
    """Spatial pyramid pooling - fast (reference block.py:177-196)."""

    def __init__(self, c1, c2, k=5):
        super().__init__()
        c_ = c1 // 2
        self.cv1 = Conv(c1, c_, 1, 1)
        self.cv2 = Conv(c_ * 4, c2, 1, 1)
        self.k = k

    def forward(self, x):
        y = [self.cv1(x)]
        for _ in range(3):
            y.append(K.maxpool(y[-1], self.k))
        return self.cv2(K.cat(y))


class MLCA(nn.Module):
    """Mixed local channel attention (reference block.py:1540-1584). Parameters: conv, conv_local (1,1,k)."""

    def __init__(self, in_size, local_size=5, gamma=2, b=1, local_weight=0.5):
        super().__init__()
        if local_size != 5:
            raise NotImplementedError("libadr MLCA kernels are built for local_size=5 (the reference default)")
        self.local_size, self.gamma, self.b = local_size, gamma, b
        t = int(abs(math.log(in_size, 2) + self.b) / self.gamma)
        k = t if t % 2 else t + 1
        self.conv = nn.Conv1d(1, 1, kernel_size=k, padding=(k - 1) // 2, bias=False)
        self.conv_local = nn.Conv1d(1, 1, kernel_size=k, padding=(k - 1) // 2, bias=False)
        self.local_weight = local_weight

    def forward(self, x, res=None):
        return K.mlca(x, res, self.conv_local.weight, self.conv.weight, self.local_weight)


class Bottleneck_MLCA(Bottleneck):
    """Bottleneck with MLCA on the residual branch (reference block.py:1586-1594); residual add fused."""

    def __init__(self, c1, c2, shortcut=True, g=1, k=(3, 3), e=0.5):
        super().__init__(c1, c2, shortcut, g, k, e)
        self.attention = MLCA(c2)

    def forward(self, x):
        y = self.cv2(self.cv1(x))
        return self.attention(y, x if self.add else None)


class C3k_MLCA(C3k):
    """Reference block.py:1596-1600."""

    def __init__(self, c1, c2, n=1, shortcut=False, g=1, e=0.5, k=3):
        super().__init__(c1, c2, n, shortcut, g, e, k)
        c_ = int(c2 * e)
        self.m = nn.Sequential(*(Bottleneck_MLCA(c_, c_, shortcut, g, k=(k, k), e=1.0) for _ in range(n)))


class C3k2_MLCA(C3k2):
    """Reference block.py:1602-1605."""

    def __init__(self, c1, c2, n=1, c3k=False, e=0.5, g=1, shortcut=True):
        super().__init__(c1, c2, n, c3k, e, g, shortcut)
        self.m = nn.ModuleList(C3k_MLCA(self.c, self.c, 2, shortcut, g) if c3k else
                               Bottleneck_MLCA(self.c, self.c, shortcut, g) for _ in range(n))


class ELA_HSFPN(nn.Module):  # noqa: N801 (reference name)
    """Efficient local attention gate (reference block.py:1408-1424): row/column means -> shared
    Conv1d(C, C, 7, p=3) -> GroupNorm(16) -> sigmoid -> x * a_h * a_w (flag) or a_h * a_w."""

    def __init__(self, in_planes, flag=True):
        super().__init__()
        self.conv1x1 = nn.Sequential(nn.Conv1d(in_planes, in_planes, 7, padding=3), nn.GroupNorm(16, in_planes),
                                     nn.Sigmoid())
        self.flag = flag

    def forward(self, x):
        N, C, H, W = x.shape
        conv, gn = self.conv1x1[0], self.conv1x1[1]
        p = K.axis_mean(x, "ela")  # (2N, C, L, 1): both branches as separate "images" (GN per branch)
        w4 = conv.weight.unsqueeze(-1)  # (C, C, 7) -> (C, C, 7, 1): a 7x1 conv over the pooled axis
        y, _ = K.conv2d(p, w4, conv.bias, (1, 1), (3, 0))
        a = K.gn_act(y, gn, "sigmoid")
        return K.gate(x if self.flag else None, a, a, "ela", x.shape)


class Multiply(nn.Module):
    """x[0] * x[1] (reference block.py:1442-1447)."""

    def forward(self, x):
        return K.mul(x[0], x[1])


class Add(nn.Module):
    """sum(stack(x)) (reference block.py:1448-1453)."""

    def forward(self, x):
        if len(x) == 2:
            return K.add(x[0], x[1])
        if len(x) == 3:
            return K.add(x[0], x[1], x[2])
        out = K.add(x[0], x[1])
        for t in x[2:]:
            out = K.add(out, t)
        return out


class Fusion(nn.Module):
    """BiFPN fusion (reference block.py:1500-1537); only fusion='bifpn' is on the AD-Refine path."""

    def __init__(self, inc_list, fusion="bifpn"):
        super().__init__()
        if fusion != "bifpn":
            raise NotImplementedError(f"Fusion('{fusion}') is not on the AD-Refine hot path")
        self.fusion = fusion
        self.fusion_weight = nn.Parameter(torch.ones(len(inc_list), dtype=torch.float32), requires_grad=True)
        self.epsilon = 1e-4

    def forward(self, x):
        return K.fusion(self.fusion_weight, list(x))


class DFL(nn.Module):
    """Distribution focal loss integral (reference block.py:63-81); frozen arange weights. Applied inside the
    fused detect-decode kernel; this module holds the parameter so state_dict keys match."""

    def __init__(self, c1=16):
        super().__init__()
        self.conv = nn.Conv2d(c1, 1, 1, bias=False).requires_grad_(False)
        self.conv.weight.data[:] = torch.arange(c1, dtype=torch.float).view(1, c1, 1, 1)
        self.c1 = c1
