"""Restatement of mmcv.ops.ModulatedDeformConv2d (DCNv2) in plain PyTorch, CPU, for the oracle.

mmcv's published algorithm (modulated_deform_conv, `modulated_deformable_im2col` +
`dmcn_im2col_bilinear`): for output pixel (h, w) and tap k=(i, j) of a kh x kw kernel,
  offset channel 2k   -> dy, channel 2k+1 -> dx (deform_groups=1), mask channel k -> m;
  sample point  (py, px) = (h*s - p + i*d + dy, w*s - p + j*d + dx);
  value = 0 if py <= -1 or px <= -1 or py >= H or px >= W, else bilinear interpolation whose four
  corners are each bounds-checked (a corner outside [0,H)x[0,W) contributes 0);
  column = value * m;  out = W[Cout, Cin*kh*kw] @ columns (+ bias).
Gradients follow by autograd through the same arithmetic (mmcv's analytic backward computes the same
derivatives). Oracle / fixture generation only.
"""
import math

import torch
import torch.nn as nn


def modulated_deform_conv2d(x, offset, mask, weight, bias, stride=1, padding=1, dilation=1):
    B, C, H, W = x.shape
    Cout, Cin, KH, KW = weight.shape
    Ho = (H + 2 * padding - (dilation * (KH - 1) + 1)) // stride + 1
    Wo = (W + 2 * padding - (dilation * (KW - 1) + 1)) // stride + 1
    dev, dt = x.device, x.dtype
    hs = (torch.arange(Ho, device=dev, dtype=dt) * stride - padding).view(1, Ho, 1)
    ws = (torch.arange(Wo, device=dev, dtype=dt) * stride - padding).view(1, 1, Wo)
    xf = x.reshape(B, C, H * W)
    cols = []
    for i in range(KH):
        for j in range(KW):
            k = i * KW + j
            py = hs + i * dilation + offset[:, 2 * k]
            px = ws + j * dilation + offset[:, 2 * k + 1]
            valid = (py > -1) & (px > -1) & (py < H) & (px < W)
            y0 = torch.floor(py)
            x0 = torch.floor(px)
            ly = py - y0
            lx = px - x0
            hy = 1 - ly
            hx = 1 - lx
            y0i = y0.long()
            x0i = x0.long()
            val = torch.zeros(B, C, Ho, Wo, device=dev, dtype=dt)
            for dy, dx, wgt in ((0, 0, hy * hx), (0, 1, hy * lx), (1, 0, ly * hx), (1, 1, ly * lx)):
                yy = y0i + dy
                xx = x0i + dx
                ok = valid & (yy >= 0) & (yy < H) & (xx >= 0) & (xx < W)
                idx = (yy.clamp(0, H - 1) * W + xx.clamp(0, W - 1)).view(B, 1, Ho * Wo).expand(B, C, Ho * Wo)
                g = torch.gather(xf, 2, idx).view(B, C, Ho, Wo)
                val = val + g * (wgt * ok.to(dt)).unsqueeze(1)
            cols.append(val * mask[:, k].unsqueeze(1))
    col = torch.stack(cols, 2).reshape(B, C * KH * KW, Ho * Wo)
    out = torch.matmul(weight.reshape(Cout, -1), col).view(B, Cout, Ho, Wo)
    if bias is not None:
        out = out + bias.view(1, -1, 1, 1)
    return out


class ModulatedDeformConv2d(nn.Module):
    def __init__(self, in_channels, out_channels, kernel_size, stride=1, padding=0, dilation=1, groups=1,
                 deform_groups=1, bias=True):
        super().__init__()
        assert groups == 1 and deform_groups == 1
        k = kernel_size if isinstance(kernel_size, int) else kernel_size[0]
        self.in_channels, self.out_channels = in_channels, out_channels
        self.kernel_size = (k, k)
        self.stride, self.padding, self.dilation = stride, padding, dilation
        self.weight = nn.Parameter(torch.empty(out_channels, in_channels, k, k))
        if bias:
            self.bias = nn.Parameter(torch.zeros(out_channels))
        else:
            self.register_parameter("bias", None)
        n = in_channels * k * k
        stdv = 1.0 / math.sqrt(n)
        self.weight.data.uniform_(-stdv, stdv)

    def forward(self, x, offset, mask):
        return modulated_deform_conv2d(x, offset, mask, self.weight, self.bias, self.stride, self.padding,
                                       self.dilation)
