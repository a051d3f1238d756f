"""Detection heads — HIP-backed drop-ins for the reference's ultralytics/nn/modules/head.py with identical
class names, constructor signatures and parameter names (state_dict keys): the stock YOLOv8/11 Detect
(head.py:21-161) and AYHead (alias of AYHead1) with its parts (head.py:600-1252). Output contract (head.py:61-70,
1178-1204): train -> list of (B, no, H, W); eval -> (y (B, 4+nc, A) fp32, list) or y when `export`.
"""
from __future__ import annotations

import math

import torch
import torch.nn as nn

from ... import kernels as K
from .block import DFL
from .conv import Conv, Conv2d, DWConv, autopad

__all__ = ("Detect", "Conv_GN", "TaskDecomposition", "CoordAtt", "CrossTaskInteraction", "DyDCNv2", "Scale", "ResidualBlockGN",
           "AYHead1", "AYHead")


class Detect(nn.Module):
    """YOLOv8/11 Detect head (head.py:21-161): per level a box branch (two 3x3 Conv, a 1x1 nn.Conv2d to
    4*reg_max) and a class branch (DWConv 3x3 + Conv 1x1, twice, then a 1x1 nn.Conv2d to nc), concatenated
    channel-wise. Eval decodes with the fused DFL + dist2bbox + sigmoid kernel (_inference, head.py:86-115).
    end2end (YOLOv10) is not part of this build."""

    dynamic = False
    export = False
    end2end = False
    max_det = 300
    shape = None
    anchors = torch.empty(0)
    strides = torch.empty(0)
    format = None

    def __init__(self, nc=80, ch=()):
        super().__init__()
        self.nc = nc
        self.nl = len(ch)
        self.reg_max = 16
        self.no = nc + self.reg_max * 4
        self.stride = torch.zeros(self.nl)
        c2, c3 = max((16, ch[0] // 4, self.reg_max * 4)), max(ch[0], min(self.nc, 100))
        self.cv2 = nn.ModuleList(
            nn.Sequential(Conv(x, c2, 3), Conv(c2, c2, 3), Conv2d(c2, 4 * self.reg_max, 1)) for x in ch)
        self.cv3 = nn.ModuleList(
            nn.Sequential(nn.Sequential(DWConv(x, x, 3), Conv(x, c3, 1)),
                          nn.Sequential(DWConv(c3, c3, 3), Conv(c3, c3, 1)),
                          Conv2d(c3, self.nc, 1)) for x in ch)
        self.dfl = DFL(self.reg_max) if self.reg_max > 1 else nn.Identity()

    def forward(self, x):
        out = []
        for i in range(self.nl):
            xa, xb = K.fanout(x[i])  # the level feature feeds both branches: one HIP gradient sum
            out.append(K.cat([self.cv2[i](xa), self.cv3[i](xb)]))
        if self.training:
            return out
        if self.nl != 3:
            raise NotImplementedError("adrefine Detect: the fused decode handles 3 levels (P3-P5)")
        y = K.detect_decode(out, [float(s) for s in self.stride], self.nc, self.reg_max)
        return y if self.export else (y, out)

    def bias_init(self):
        """head.py:137-147: box bias 1.0, class bias log(5 / nc / (640 / s)^2) (0.01 objects per 640 image)."""
        for a, b, s in zip(self.cv2, self.cv3, self.stride):
            a[-1].bias.data[:] = 1.0
            b[-1].bias.data[: self.nc] = math.log(5 / self.nc / (640 / float(s)) ** 2)


class Conv_GN(nn.Module):  # noqa: N801
    """Conv2d(no bias) -> GroupNorm(16) -> SiLU (head.py:607-620)."""

    default_act = "silu"

    def __init__(self, c1, c2, k=1, s=1, p=None, g=1, d=1, act=True):
        super().__init__()
        self.conv = Conv2d(c1, c2, k, s, autopad(k, p, d), groups=g, dilation=d, bias=False)
        self.gn = nn.GroupNorm(16, c2)
        self.act_name = "silu" if act is True else ("none" if act is False else act)

    def forward(self, x, pack=None):
        """pack: x is a level-packed activation (AYHead1): GroupNorm per (level, image), k x k convs per level."""
        if pack is None:
            y, _ = K.conv2d(x, self.conv.weight, None, self.conv.stride[0], self.conv.padding[0])
            return K.gn_act(y, self.gn, self.act_name)
        if self.conv.stride[0] != 1 or self.conv.groups != 1:
            raise NotImplementedError("packed Conv_GN: stride 1, dense")
        if self.conv.kernel_size[0] == 1:
            y, _ = K.conv2d(x, self.conv.weight, None, 1, 0)
        else:
            y = K.level_conv(x, self.conv.weight, None, self.conv.padding[0], pack)
        return K.gn_act_packed(y, pack, [self.gn], self.act_name)


class TaskDecomposition(nn.Module):
    """Layer-attention gated 1x1 (head.py:626-669). With stacked_convs=1 the gate is one scalar per image, so
    conv(feat, s_b * W) == s_b * conv(feat, W): run the shared 1x1 on the MFMA engine and scale per image."""

    def __init__(self, feat_channels, stacked_convs, la_down_rate=8):
        super().__init__()
        self.feat_channels = feat_channels
        self.stacked_convs = stacked_convs
        self.in_channels = feat_channels * stacked_convs
        self.la_conv1 = nn.Conv2d(self.in_channels, self.in_channels // la_down_rate, 1)
        self.relu = nn.ReLU(inplace=True)
        self.la_conv2 = nn.Conv2d(self.in_channels // la_down_rate, self.stacked_convs, 1, padding=0)
        self.sigmoid = nn.Sigmoid()
        self.reduction_conv = Conv_GN(self.in_channels, self.feat_channels, 1)
        nn.init.normal_(self.la_conv1.weight.data, mean=0, std=0.001)
        nn.init.normal_(self.la_conv2.weight.data, mean=0, std=0.001)
        nn.init.zeros_(self.la_conv2.bias.data)
        nn.init.normal_(self.reduction_conv.conv.weight.data, mean=0, std=0.01)

    def forward(self, feat, avg_feat=None, pack=None):
        if self.stacked_convs != 1:
            raise NotImplementedError("AYHead uses TaskDecomposition(stacked_convs=1)")
        if avg_feat is None:
            avg_feat = K.gap(feat) if pack is None else K.gap_packed(feat, pack)
        s = K.gate_mlp(avg_feat, self.la_conv1.weight, self.la_conv1.bias, self.la_conv2.weight, self.la_conv2.bias,
                       "relu", "sigmoid")  # (N, 1)
        y, _ = K.conv2d(feat, self.reduction_conv.conv.weight, None, 1, 0)
        s = s.view(-1) if pack is None else K.seg_expand(s.view(-1), pack)  # packed: the image's gate per sub-image
        y = K.scale(y, s, "n", grad_from_out=True)  # GroupNorm follows: d/ds from the GN input itself
        if pack is not None:
            return K.gn_act_packed(y, pack, [self.reduction_conv.gn], "silu")
        return K.gn_act(y, self.reduction_conv.gn, "silu")


class CoordAtt(nn.Module):
    """Coordinate attention (head.py:671-707)."""

    def __init__(self, inp, oup, reduction=32):
        super().__init__()
        mip = max(8, inp // reduction)
        self.conv1 = Conv2d(inp, mip, kernel_size=1, stride=1, padding=0)
        self.bn1 = nn.BatchNorm2d(mip, eps=1e-3, momentum=0.03)  # initialize_weights (torch_utils.py:430-432)
        self.act = nn.Hardswish()
        self.conv_h = Conv2d(mip, oup, kernel_size=1, stride=1, padding=0)
        self.conv_w = Conv2d(mip, oup, kernel_size=1, stride=1, padding=0)

    def _attn(self, y, pp=None):
        y, _ = K.conv2d(y, self.conv1.weight, self.conv1.bias, 1, 0)
        if pp is not None and self.training:  # the levels' planes in one tensor: BatchNorm statistics per level
            y = K.bn_act_packed(y, pp, self.bn1, "hswish")
        else:
            y = K.bn_act(y, None, self.bn1, "hswish", self.training)
        a_h = K.conv_act(y, self.conv_h.weight, self.conv_h.bias, 1, 0, "sigmoid")
        a_w = K.conv_act(y, self.conv_w.weight, self.conv_w.bias, 1, 0, "sigmoid")
        return a_h, a_w

    def forward(self, x, pack=None):
        x, xg = K.fanout(x)
        if pack is None:
            a_h, a_w = self._attn(K.axis_mean(x, "coord"))  # (N, C, H+W, 1): [row means ; column means]
            return K.gate(xg, a_h, a_w, "coord", x.shape)
        # packed: every level's pooled plane in one tensor (conv1 / BN / conv_h / conv_w once), gates per level
        pp = K.LevelPack(pack.N, [(1, h + w) for h, w in pack.dims])
        a_h, a_w = self._attn(K.axis_mean_levels(x, pack, pp), pp)
        return K.gate_levels(xg, a_h, a_w, pack, pp)


class CrossTaskInteraction(nn.Module):
    """head.py:722-747."""

    def __init__(self, channels):
        super().__init__()
        self.cls_to_reg = Conv2d(channels, channels, 1)
        self.reg_to_cls = Conv2d(channels, channels, 1)
        self.cls_gate = nn.Sequential(Conv2d(channels * 2, channels, 1), nn.Sigmoid())
        self.reg_gate = nn.Sequential(Conv2d(channels * 2, channels, 1), nn.Sigmoid())

    def forward(self, cls_feat, reg_feat):
        cf = list(K.fanout(cls_feat, 3))
        rf = list(K.fanout(reg_feat, 3))
        # the gates' concat inputs: the cross convs write their halves in place (one copy per concat, not two)
        N, C, H, W = cls_feat.shape
        bc = K.empty_act(N, 2 * C, H, W, cls_feat.dtype, cls_feat.device)
        br = K.empty_act(N, 2 * C, H, W, reg_feat.dtype, reg_feat.device)
        c2r = list(K.fanout(self.cls_to_reg(cf[0], out=br[:, C:])))
        r2c = list(K.fanout(self.reg_to_cls(rf[0], out=bc[:, C:])))
        g0, h0 = self.cls_gate[0], self.reg_gate[0]
        cg = K.conv_act(K.cat([cf[1], r2c[0]], out=bc), g0.weight, g0.bias, 1, 0, "sigmoid")
        rg = K.conv_act(K.cat([rf[1], c2r[0]], out=br), h0.weight, h0.bias, 1, 0, "sigmoid")
        return K.fma(cf[2], r2c[1], cg), K.fma(rf[2], c2r[1], rg)


class _DCNWeight(nn.Module):
    """Parameter holder with mmcv ModulatedDeformConv2d's names (weight; bias absent when a norm follows)."""

    def __init__(self, cin, cout, k=3):
        super().__init__()
        self.in_channels, self.out_channels, self.kernel_size = cin, cout, (k, k)
        self.weight = nn.Parameter(torch.empty(cout, cin, k, k))
        self.register_parameter("bias", None)
        nn.init.uniform_(self.weight, -1.0 / math.sqrt(cin * k * k), 1.0 / math.sqrt(cin * k * k))


class DyDCNv2(nn.Module):
    """ModulatedDeformConv2d(3x3, s1, p1, no bias) + GroupNorm(16) (head.py:751-782)."""

    def __init__(self, in_channels, out_channels, stride=1, norm_cfg=None):
        super().__init__()
        if stride != 1:
            raise NotImplementedError("DyDCNv2 stride != 1 is not on the AYHead path")
        self.with_norm = True
        self.conv = _DCNWeight(in_channels, out_channels)
        self.norm = nn.GroupNorm(16, out_channels)

    def forward(self, x, om, pack=None):
        """`om`: the spatial_conv_offset output (offsets [0,18) and mask LOGITS [18,27); sigmoid fused)."""
        if pack is not None:
            return K.gn_act_packed(K.dcn_levels(x, om, self.conv.weight, pack), pack, [self.norm], "none")
        return K.gn_act(K.dcn(x, om, self.conv.weight), self.norm, "none")


class Scale(nn.Module):
    """Learnable scalar (head.py:785-798)."""

    def __init__(self, scale: float = 1.0):
        super().__init__()
        self.scale = nn.Parameter(torch.tensor(scale, dtype=torch.float))

    def forward(self, x, out=None):
        return K.scale(x, self.scale, "scalar", out=out)


class ResidualBlockGN(nn.Module):
    """head.py:1031-1047."""

    def __init__(self, c1, c2, k=3, s=1, p=None, act=True):
        super().__init__()
        self.conv1 = Conv_GN(c1, c2, k, s, p=p, act=act)
        self.conv2 = Conv_GN(c2, c2, k, s, p=p, act=act)
        self.shortcut = nn.Identity() if c1 == c2 and s == 1 else Conv_GN(c1, c2, 1, s, act=False)

    def forward(self, x, pack=None):
        x, xs = K.fanout(x)
        res = xs if isinstance(self.shortcut, nn.Identity) else self.shortcut(xs, pack)
        return K.add(self.conv2(self.conv1(x, pack), pack), res)


class AYHead1(nn.Module):
    """AD-Refine detection head (head.py:1049-1252)."""

    dynamic = False
    export = False
    shape = None
    anchors = torch.empty(0)
    strides = torch.empty(0)
    format = None

    def __init__(self, nc=80, ch=()):
        super().__init__()
        self.nc = nc
        self.nl = len(ch)
        self.reg_max = 16
        self.no = nc + self.reg_max * 4
        self.stride = torch.zeros(self.nl)
        self.ch = ch
        hidc = max(ch) if ch else 512
        task_ch = hidc // 2
        self.stems = nn.ModuleList(Conv_GN(self.ch[i], hidc, 1) for i in range(self.nl))
        self.share_conv = nn.Sequential(Conv_GN(hidc, task_ch, 3), Conv_GN(task_ch, task_ch, 3))
        self.cls_decomp = TaskDecomposition(feat_channels=task_ch, stacked_convs=1, la_down_rate=16)
        self.reg_decomp = TaskDecomposition(feat_channels=task_ch, stacked_convs=1, la_down_rate=16)
        self.rep_block_cls = ResidualBlockGN(task_ch, task_ch)
        self.coord_attention_reg = CoordAtt(task_ch, task_ch)
        self.cross_task = CrossTaskInteraction(task_ch)
        self.spatial_conv_offset = Conv2d(task_ch, 3 * 3 * 3, 3, padding=1)
        self.offset_dim = 2 * 3 * 3
        self.DyDCNV2 = DyDCNv2(task_ch, task_ch)
        self.cls_prob_conv = nn.Sequential(Conv2d(task_ch, task_ch // 2, 1), nn.ReLU(),
                                           Conv2d(task_ch // 2, 1, 3, padding=1), nn.Sigmoid())
        self.cv2 = Conv2d(task_ch, 4 * self.reg_max, 1)
        self.cv3 = Conv2d(task_ch, self.nc, 1)
        self.scale = nn.ModuleList([Scale(1.0) for _ in range(self.nl)])
        self.dfl = DFL(self.reg_max) if self.reg_max > 1 else nn.Identity()
        self.initialize_biases()

    def _level(self, x, i):
        ax = self.stems[i](x)
        # feat feeds five consumers: its gradient is summed by libadr (K.fanout), not by autograd adds
        fv = list(K.fanout(self.share_conv(ax), 5))
        avg = K.gap(fv[0])
        cls_f = self.cls_decomp(fv[1], avg)
        reg_f = self.reg_decomp(fv[2], avg)
        cls_f, reg_f = self.cross_task(cls_f, reg_f)
        cls_e = self.rep_block_cls(cls_f)
        so = self.spatial_conv_offset
        om = K.padded_conv2d(fv[3], so.weight, so.bias, 1, 1, 32)  # 27 channels padded to 32
        r = self.DyDCNV2(reg_f, om)
        r = self.coord_attention_reg(r)
        c0, c2 = self.cls_prob_conv[0], self.cls_prob_conv[2]
        cp = K.conv_act(fv[4], c0.weight, c0.bias, 1, 0, "relu")
        cp = K.act(K.padded_conv2d(cp, c2.weight, c2.bias, 1, 1, 8), "sigmoid")  # channel 0 valid
        # both halves of the level's output row written in place into one buffer (no concat copies)
        N, _, H, W = r.shape
        buf = K.empty_act(N, 4 * self.reg_max + self.nc, H, W, r.dtype, r.device)
        reg_out = self.scale[i](self.cv2(r), out=buf[:, :4 * self.reg_max])
        cls_out = self.cv3(K.mul_pixel(cls_e, cp), out=buf[:, 4 * self.reg_max:])
        return K.cat([reg_out, cls_out], out=buf)

    def _packed(self, xs):
        """All levels at once in the packed row space (kernels.LevelPack): the per-pixel ops are one launch for the
        three levels, per-image statistics go through the segment kernels, 3x3 convs / DCN / CoordAtt's pooling run
        per level on views. Same math as _level per level (per-level stems / Scale, shared everything else)."""
        pack = K.LevelPack(xs[0].shape[0], [(x.shape[2], x.shape[3]) for x in xs])
        dtype, dev = xs[0].dtype, xs[0].device
        hid = self.stems[0].conv.out_channels
        sb = pack.empty(hid, dtype, dev)  # the stems write their level views in place
        ys = [K.conv2d(x, st.conv.weight, None, 1, 0, out=pack.view(sb, i))[0] for i, (x, st) in
              enumerate(zip(xs, self.stems))]
        ax = K.gn_act_packed(K.level_join(ys, pack, out=sb), pack, [st.gn for st in self.stems], "silu")
        fv = list(K.fanout(self.share_conv[1](self.share_conv[0](ax, pack), pack), 5))
        avg = K.gap_packed(fv[0], pack)
        cls_f = self.cls_decomp(fv[1], avg, pack)
        reg_f = self.reg_decomp(fv[2], avg, pack)
        cls_f, reg_f = self.cross_task(cls_f, reg_f)
        cls_e = self.rep_block_cls(cls_f, pack)
        so = self.spatial_conv_offset
        om = K.level_conv(fv[3], so.weight, so.bias, 1, pack, kpad=32)  # 27 channels padded to 32
        r = self.coord_attention_reg(self.DyDCNV2(reg_f, om, pack), pack)
        c0, c2 = self.cls_prob_conv[0], self.cls_prob_conv[2]
        cp = K.conv_act(fv[4], c0.weight, c0.bias, 1, 0, "relu")
        cp = K.act(K.level_conv(cp, c2.weight, c2.bias, 1, pack, kpad=8), "sigmoid")  # channel 0 valid
        buf = pack.empty(4 * self.reg_max + self.nc, dtype, dev)
        reg_out = K.scale_levels(self.cv2(r), [s.scale for s in self.scale], pack, out=buf[:, :4 * self.reg_max])
        cls_out = self.cv3(K.mul_pixel(cls_e, cp), out=buf[:, 4 * self.reg_max:])
        return list(K.level_split(K.cat([reg_out, cls_out], out=buf), pack))

    # the packed head (one pass over all levels) is the default; False runs the reference's per-level loop
    # (tests compare the two)
    packed = True

    def forward(self, x):
        if self.packed and len(x) > 1:
            outputs = self._packed(list(x))
        else:  # the reference loops the levels (head.py:1132)
            outputs = [self._level(xi, i) for i, xi in enumerate(x)]
        if self.training:
            return outputs
        y = K.detect_decode(outputs, [float(s) for s in self.stride], self.nc, self.reg_max)
        return y if self.export else (y, outputs)

    def initialize_biases(self):
        """head.py:1206-1228: default strides [8, 16, 32], cv2 bias 1.0, cv3 bias prior 0.01."""
        if (self.stride == 0).all():
            self.stride = torch.tensor([8, 16, 32, 64, 128][: self.nl], dtype=torch.float32)
        self.cv2.bias.data.fill_(1.0)
        self.cv3.bias.data.fill_(-math.log((1 - 0.01) / 0.01))

    def bias_init(self):
        self.initialize_biases()


AYHead = AYHead1
