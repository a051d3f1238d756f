"""Convolution modules — HIP-backed drop-ins for the reference's ultralytics/nn/modules/conv.py.

Class names, constructor signatures and parameter names match the reference so yaml configs and
state_dicts load unchanged; forward passes run libadr_hip kernels on NHWC (channels_last) activations.
"""
from __future__ import annotations

import math

import torch
import torch.nn as nn

from ... import kernels as K

__all__ = ("Conv", "DWConv", "Conv2d", "ConvTranspose2d", "Concat", "Upsample", "autopad")


def autopad(k, p=None, d=1):
    """Pad to 'same' output (reference conv.py:27-33)."""
    if d > 1:
        k = d * (k - 1) + 1 if isinstance(k, int) else [d * (x - 1) + 1 for x in k]
    if p is None:
        p = k // 2 if isinstance(k, int) else [x // 2 for x in k]
    return p


def _act_name(act):
    if act is True:
        return Conv.default_act
    if act is False or act is None:
        return "none"
    if isinstance(act, str):
        return act
    name = type(act).__name__.lower()
    return {"silu": "silu", "gelu": "gelu", "relu": "relu", "sigmoid": "sigmoid", "hardswish": "hswish",
            "identity": "none"}[name]


def _in_pad(x, w):
    """The stem receives images padded to 8 channels (kernels.image_to_nhwc); pad the weight to match."""
    return x.shape[1] if x.shape[1] != w.shape[1] and w.shape[1] < 8 else 0


class Conv2d(nn.Conv2d):
    """nn.Conv2d drop-in (dense, dilation 1). Used for the yaml `nn.Conv2d` rows (tasks.py:1016)."""

    def forward(self, x, out=None):
        if self.groups != 1 or self.dilation != (1, 1) or self.stride[0] != self.stride[1] or \
                self.padding[0] != self.padding[1]:
            raise NotImplementedError("adrefine Conv2d: grouped / dilated / anisotropic convs use DWConv kernels")
        y, _ = K.conv2d(x, self.weight, self.bias, self.stride[0], self.padding[0], False, _in_pad(x, self.weight),
                        out=out)
        return y


class ConvTranspose2d(nn.ConvTranspose2d):
    """nn.ConvTranspose2d drop-in (yaml L13/L20: 128->128, k3 s2 p1 op1)."""

    def forward(self, x, output_size=None):
        if self.groups != 1 or self.dilation != (1, 1):
            raise NotImplementedError("adrefine ConvTranspose2d: groups/dilation unsupported")
        return K.conv_transpose2d(x, self.weight, self.bias, self.stride[0], self.padding[0], self.output_padding[0])


class Conv(nn.Module):
    """Conv2d(no bias) -> BatchNorm2d -> SiLU (reference conv.py:36-54), fused on the GPU:
    implicit-GEMM conv with BN partial statistics in the epilogue, then normalise + activation. Depthwise
    instances (g == c1 == c2: DWConv, Attention.pe) run the depthwise kernel instead of the GEMM."""

    default_act = "silu"

    def __init__(self, c1, c2, k=1, s=1, p=None, g=1, d=1, act=True):
        super().__init__()
        self.conv = Conv2d(c1, c2, k, s, autopad(k, p, d), groups=g, dilation=d, bias=False)
        self.bn = nn.BatchNorm2d(c2, eps=1e-3, momentum=0.03)  # initialize_weights (torch_utils.py:430-432)
        self.act_name = _act_name(act)

    accepts_out = True  # forward(x, out=view) writes the activation into a caller's concat slice

    def forward(self, x, out=None, lazy=False, res=None):
        """lazy (training): the caller hands the output straight to a conv, which applies this BN-act while staging
        it (kernels.BnFwd) — the output is written by that conv, not by an elementwise pass here. res: a residual
        added to the output (Bottleneck's shortcut) — in the BN-act pass when training, else one add."""
        if res is not None and not (self.training and self.conv.groups == 1):
            return K.add(res, self.forward(x, lazy=lazy), out=out)
        cv = self.conv
        if cv.groups != 1:
            k = cv.kernel_size[0]
            if not (cv.groups == cv.in_channels == cv.out_channels and cv.stride == (1, 1) and cv.dilation == (1, 1)
                    and cv.kernel_size == (k, k) and cv.padding == (k // 2, k // 2)):
                raise NotImplementedError("adrefine Conv: grouped convs are depthwise, stride 1, 'same' padding")
            if not self.training and K.EVAL_CONV_BN_ACT:  # inference: BN + act in the depthwise kernel
                z = K.dwconv_bn_act_eval(x, cv.weight, k, self.bn, self.act_name, out=out)
                if z is not None:
                    return z
            return K.bn_act(K.dwconv(x, cv.weight, None, k), None, self.bn, self.act_name, self.training, out=out)
        if not self.training and K.EVAL_CONV_BN_ACT:  # inference: BN + act in the conv epilogue (forward_fuse)
            z = K.conv_bn_act_eval(x, cv.weight, cv.stride[0], cv.padding[0], self.bn, self.act_name,
                                   _in_pad(x, cv.weight), out=out)
            if z is not None:
                return z
        # training: BN partial statistics in the conv epilogue, then finalize + affine + act (or, lazily, the
        # consumer conv applies the affine + act while staging)
        y, st = K.conv2d(x, cv.weight, None, cv.stride[0], cv.padding[0], self.training, _in_pad(x, cv.weight))
        return K.bn_act(y, st, self.bn, self.act_name, self.training, out=out, xfuse=True, lazy=lazy and out is None,
                        res=res)

    def stem_ok(self):
        """The adr_stem kernels cover Conv(3, K in {16, 32, 64}, 3, 2) with pad 1 (every yaml's model.0)."""
        cv = self.conv
        return (cv.in_channels == 3 and cv.out_channels in (16, 32, 64) and cv.kernel_size == (3, 3)
                and cv.stride == (2, 2) and cv.padding == (1, 1) and cv.groups == 1 and cv.dilation == (1, 1))

    def forward_image(self, img, lazy=False):
        """The same Conv on the fp32 NCHW image batch, through the stem kernels (bf16 compute). lazy: as forward."""
        y, st = K.stem_conv(img, self.conv.weight, self.training)
        return K.bn_act(y, st if st.numel() else None, self.bn, self.act_name, self.training, lazy=lazy)


class DWConv(Conv):
    """Depth-wise convolution (reference conv.py:101-106): Conv with g = gcd(c1, c2)."""

    def __init__(self, c1, c2, k=1, s=1, d=1, act=True):
        super().__init__(c1, c2, k, s, g=math.gcd(c1, c2), d=d, act=act)


class Concat(nn.Module):
    """torch.cat(x, dim) (reference conv.py:322-335); channel concatenation of NHWC activations."""

    def __init__(self, dimension=1):
        super().__init__()
        self.d = dimension

    def forward(self, x):
        if self.d != 1:
            raise NotImplementedError("adrefine Concat: channel (dim 1) concatenation only")
        return K.cat(list(x))


class Upsample(nn.Upsample):
    """nn.Upsample drop-in for the yaml `nn.Upsample, [None, s, 'nearest']` rows (integer factor)."""

    def forward(self, x):
        sf = self.scale_factor
        sf = sf[0] if isinstance(sf, tuple) else sf
        if self.mode != "nearest" or self.size is not None or sf is None or float(sf) != int(sf):
            raise NotImplementedError("adrefine Upsample: nearest mode with an integer scale_factor")
        return K.upsample_nearest(x, int(sf))
