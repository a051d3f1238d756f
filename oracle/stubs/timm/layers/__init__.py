import math

import torch
import torch.nn as nn


class DropPath(nn.Module):
    def __init__(self, drop_prob=0.0, scale_by_keep=True):
        super().__init__()
        self.drop_prob = drop_prob

    def forward(self, x):
        return x


def trunc_normal_(tensor, mean=0.0, std=1.0, a=-2.0, b=2.0):
    with torch.no_grad():
        return nn.init.trunc_normal_(tensor, mean, std, a, b)


def to_2tuple(x):
    return tuple(x) if isinstance(x, (list, tuple)) else (x, x)


def drop_path(x, drop_prob=0.0, training=False, scale_by_keep=True):
    return x


_ = math
