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
from .mona import Mona

__all__ = ("Bottleneck", "C2f", "C3", "C3k", "C3k2", "SPPF", "MLCA", "Bottleneck_MLCA", "C3k_MLCA", "C3k2_MLCA",
           "ELA_HSFPN", "Multiply", "Add", "Fusion", "DFL", "Attention", "PSABlock", "C2PSA", "C2PTSSA", "DynamicTanh", "AttentionTSSA",
           "TSSAlock_DYT_Mona_EDFFN", "C2TSSA_DYT_Mona_EDFFN")


class Bottleneck(nn.Module):
    """Standard bottleneck (reference block.py:341-354)."""

    def __init__(self, c1, c2, shortcut=True, g=1, k=(3, 3), e=0.5):
        super().__init__()
        c_ = int(c2 * e)
        self.cv1 = Conv(c1, c_, k[0], 1)
        self.cv2 = Conv(c_, c2, k[1], 1, g=g)
        self.add = shortcut and c1 == c2

    accepts_out = True

    def forward(self, x, out=None):
        if self.add:
            xa, xb = K.fanout(x)  # residual + branch: one HIP gradient sum instead of an autograd add
            return self.cv2(self.cv1(xb, lazy=True), out=out, res=xa)  # the add in cv2's BN-act pass
        return self.cv2(self.cv1(x, lazy=True), out=out)


class C2f(nn.Module):
    """CSP bottleneck with 2 convolutions (reference block.py:232-247)."""

    def __init__(self, c1, c2, n=1, shortcut=False, g=1, e=0.5):
        super().__init__()
        self.c = int(c2 * e)
        self.cv1 = Conv(c1, 2 * self.c, 1, 1)
        self.cv2 = Conv((2 + n) * self.c, c2, 1)
        self.m = nn.ModuleList(Bottleneck(self.c, self.c, shortcut, g, k=((3, 3), (3, 3)), e=1.0) for _ in range(n))

    def forward(self, x, lazy=False):
        # cv1 and every block that can write its output through an `out=` view write straight into their slice
        # of the concat buffer, so the concat copies only the pieces of blocks that cannot (e.g. MLCA bottlenecks).
        # lazy: the caller hands the output to a conv (its only reader) — cv2's BN-act is applied by that conv
        N, _, H, W = x.shape
        c, n = self.c, len(self.m)
        buf = K.empty_act(N, (2 + n) * c, H, W, x.dtype, x.device)
        ys = list(K.split(self.cv1(x, out=buf[:, :2 * c]), (c, c)))  # chunk(2, 1): NHWC views, no copy
        for i, m in enumerate(self.m):
            ys[-1], feed = K.fanout(ys[-1])  # used by the concat and by m: one gradient sum, in the concat slice
            slot = buf[:, (2 + i) * c:(3 + i) * c]
            ys.append(m(feed, out=slot) if getattr(m, "accepts_out", False) else m(feed))
        return self.cv2(K.cat(ys, out=buf), lazy=lazy)


class C3(nn.Module):
    """CSP bottleneck with 3 convolutions (reference block.py:256-270)."""

    def __init__(self, c1, c2, n=1, shortcut=True, g=1, e=0.5):
        super().__init__()
        c_ = int(c2 * e)
        self.cv1 = Conv(c1, c_, 1, 1)
        self.cv2 = Conv(c1, c_, 1, 1)
        self.cv3 = Conv(2 * c_, c2, 1)
        self.m = nn.Sequential(*(Bottleneck(c_, c_, shortcut, g, k=((1, 1), (3, 3)), e=1.0) for _ in range(n)))

    accepts_out = True

    def forward(self, x, out=None):
        # the last bottleneck and cv2 write straight into their halves of the concat buffer (no copies)
        xa, xb = K.fanout(x)
        N, _, H, W = x.shape
        c_ = self.cv1.conv.out_channels
        buf = K.empty_act(N, 2 * c_, H, W, x.dtype, x.device)
        *head, last = list(self.m)
        y = self.cv1(xa)
        for mm in head:
            y = mm(y)
        y = last(y, out=buf[:, :c_]) if getattr(last, "accepts_out", False) else last(y)
        return self.cv3(K.cat([y, self.cv2(xb, out=buf[:, c_:])], out=buf), out=out)


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

    def forward(self, x, lazy=False):
        # cv1 and the three pools write straight into their slices of the concat buffer (no copies); lazy: as C2f
        N, _, H, W = x.shape
        c_ = self.cv1.conv.out_channels
        buf = K.empty_act(N, 4 * c_, H, W, x.dtype, x.device)
        y = [self.cv1(x, out=buf[:, :c_])]
        for i in range(3):
            y[-1], feed = K.fanout(y[-1])
            y.append(K.maxpool(feed, self.k, out=buf[:, (i + 1) * c_:(i + 2) * c_]))
        return self.cv2(K.cat(y, out=buf), lazy=lazy)


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

    def forward(self, x, res=None, out=None):
        return K.mlca(x, res, self.conv_local.weight, self.conv.weight, self.local_weight, out=out)


class Bottleneck_MLCA(Bottleneck):
    """Bottleneck with MLCA on the residual branch (reference block.py:1586-1594); residual add fused."""

    accepts_out = True  # the fused MLCA kernel writes its output through an `out=` view (a concat slot)

    def __init__(self, c1, c2, shortcut=True, g=1, k=(3, 3), e=0.5):
        super().__init__(c1, c2, shortcut, g, k, e)
        self.attention = MLCA(c2)

    def forward(self, x, out=None):
        if not self.add:
            return self.attention(self.cv2(self.cv1(x, lazy=True)), None, out=out)
        xa, xb = K.fanout(x)
        return self.attention(self.cv2(self.cv1(xa, lazy=True)), xb, out=out)


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
        if self.flag:
            x, xg = K.fanout(x)
        p = K.axis_mean(x, "ela")  # (2N, C, L, 1): both branches as separate "images" (GN per branch)
        w4 = conv.weight.unsqueeze(-1)  # (C, C, 7) -> (C, C, 7, 1): a 7x1 conv over the pooled axis
        y, _ = K.conv2d(p, w4, conv.bias, (1, 1), (3, 0))
        a = K.gn_act(y, gn, "sigmoid")
        return K.gate(xg if self.flag else None, a, a, "ela", x.shape)


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


# ------------------------------------------------------------------------------------------------------------
# C2PTSSA (reference block.py:2376-2710)
# ------------------------------------------------------------------------------------------------------------


def _linear(x_tok, lin_w, lin_b):
    """nn.Linear over a (B, C, N, 1) NHWC token tensor as a 1x1 implicit GEMM."""
    y, _ = K.conv2d(x_tok, lin_w.unsqueeze(-1).unsqueeze(-1), lin_b, 1, 0)
    return y


class EDFFN(nn.Module):
    """Frequency-domain gated FFN (reference block.py:2376-2415)."""

    def __init__(self, dim, ffn_expansion_factor=2, bias=False):
        super().__init__()
        hidden = int(dim * ffn_expansion_factor)
        self.patch_size = 8
        self.dim = dim
        self.project_in = nn.Conv2d(dim, hidden * 2, kernel_size=1, bias=bias)
        self.dwconv = nn.Conv2d(hidden * 2, hidden * 2, kernel_size=3, stride=1, padding=1, groups=hidden * 2,
                                bias=bias)
        self.fft = nn.Parameter(torch.ones((dim, 1, 1, self.patch_size, self.patch_size // 2 + 1)))
        self.project_out = nn.Conv2d(hidden, dim, kernel_size=1, bias=bias)

    def forward(self, x):
        x, _ = K.conv2d(x, self.project_in.weight, self.project_in.bias, 1, 0)
        x = K.dwconv(x, self.dwconv.weight, self.dwconv.bias, 3)
        x1, x2 = K.split(x, (x.shape[1] // 2, x.shape[1] // 2))
        x = K.mul(K.act(x1, "gelu"), x2)
        x, _ = K.conv2d(x, self.project_out.weight, self.project_out.bias, 1, 0)
        return K.edffn_filter(x, self.fft)  # computed in fp32 inside the kernel (reference :2407 .float())


class CrossScaleAttentionTSSA(nn.Module):
    """Multi-scale TSSA + cross-scale multi-head attention (reference block.py:2417-2491)."""

    def __init__(self, dim, num_heads=8, qkv_bias=False, attn_drop=0.0, proj_drop=0.0, scales=(1, 2, 4), **kwargs):
        super().__init__()
        self.heads = num_heads
        self.scales = list(scales)
        self.dim = dim
        self.head_dim = dim // num_heads
        self.qkv_projections = nn.ModuleList([nn.Linear(dim, dim * 3, bias=qkv_bias) for _ in self.scales])
        self.cross_scale_fusion = nn.MultiheadAttention(embed_dim=dim, num_heads=num_heads, dropout=attn_drop,
                                                        batch_first=True)
        self.temps = nn.Parameter(torch.ones(len(self.scales), num_heads, 1))
        self.to_out = nn.Sequential(nn.Linear(dim, dim), nn.Dropout(proj_drop))

    def forward(self, x):
        B, C, H, W = x.shape
        qkvs = []
        xv = list(K.fanout(x, len(self.scales)))
        for s, proj in zip(self.scales, self.qkv_projections):
            x = xv.pop()
            xs = x if s == 1 else K.bilinear(K.adaptive_avg_pool(x, H // s, W // s), H, W)
            qkvs.append(_linear(K.tokens(xs), proj.weight, proj.bias))
        st = K.tssa_stack(self.temps, self.heads, qkvs)  # (B, C, S*HW, 1)
        mha = self.cross_scale_fusion
        qkv = _linear(st, mha.in_proj_weight, mha.in_proj_bias)
        o = K.attention(qkv, self.heads)
        o = _linear(o, mha.out_proj.weight, mha.out_proj.bias)
        fused = K.group_mean(o, len(self.scales))
        return _linear(fused, self.to_out[0].weight, self.to_out[0].bias)  # (B, C, HW, 1) tokens


class AdaptiveDynamicTanh(nn.Module):
    """Reference block.py:2493-2577 (channels_first)."""

    def __init__(self, normalized_shape, num_scales=3):
        super().__init__()
        if num_scales != 3:
            raise NotImplementedError("libadr ADyT kernels implement num_scales=3 (the reference default)")
        self.normalized_shape = normalized_shape
        self.num_scales = num_scales
        self.alphas = nn.Parameter(torch.linspace(0.3, 1.0, num_scales).view(1, num_scales, 1, 1))
        self.scale_weights = nn.Parameter(torch.ones(num_scales) / num_scales)  # unused by the reference forward
        self.weight = nn.Parameter(torch.ones(normalized_shape))
        self.bias = nn.Parameter(torch.zeros(normalized_shape))
        self.importance_gate = nn.Sequential(nn.AdaptiveAvgPool2d(1), nn.Conv2d(normalized_shape, normalized_shape // 4, 1),
                                             nn.ReLU(inplace=True), nn.Conv2d(normalized_shape // 4, num_scales, 1),
                                             nn.Softmax(dim=1))

    def forward(self, x):
        g1, g3 = self.importance_gate[1], self.importance_gate[3]
        xa, xb = K.fanout(x)
        imp = K.gate_mlp(K.gap(xa), g1.weight, g1.bias, g3.weight, g3.bias, "relu", "softmax")  # (N, 3)
        return K.adyt(xb, self.alphas, imp, self.weight, self.bias)


class ProgressiveFeatureFusion(nn.Module):
    """Reference block.py:2579-2630."""

    def __init__(self, dim, num_stages=3):
        super().__init__()
        self.num_stages = num_stages
        self.stages = nn.ModuleList()
        for _ in range(num_stages):
            self.stages.append(nn.ModuleDict({
                "conv": nn.Conv2d(dim, dim, 3, padding=1, groups=dim),
                "norm": nn.BatchNorm2d(dim, eps=1e-3, momentum=0.03),
                "activation": nn.GELU(),
                "channel_mix": nn.Conv2d(dim, dim, 1),
                "spatial_mix": nn.Conv2d(dim, dim, 7, padding=3, groups=dim),
            }))
        self.stage_fusion = nn.ModuleList([nn.Conv2d(dim * 2, dim, 1) for _ in range(num_stages - 1)])
        self.stage_attention = nn.Parameter(torch.ones(num_stages) / num_stages)

    def forward(self, x):
        # every multiply-read tensor is fanned out so its gradient is summed by one HIP launch, not autograd adds
        outs = []
        x, cur = K.fanout(x)  # base of the weighted sum / stage-0 input
        for i, st in enumerate(self.stages):
            last = i == self.num_stages - 1
            cv = list(K.fanout(cur, 2 if last else 3))
            t = K.dwconv(cv[0], st["conv"].weight, st["conv"].bias, 3)
            t = K.bn_act(t, None, st["norm"], "gelu", self.training)
            ta, tb = K.fanout(t)
            cm, _ = K.conv2d(ta, st["channel_mix"].weight, st["channel_mix"].bias, 1, 0)
            sm = K.dwconv(tb, st["spatial_mix"].weight, st["spatial_mix"].bias, 7)
            out = K.add(cm, sm, cv[1])
            if not last:
                out, ob = K.fanout(out)
                sf = self.stage_fusion[i]
                cur, _ = K.conv2d(K.cat([cv[2], ob]), sf.weight, sf.bias, 1, 0)
            outs.append(out)
        return K.weighted_sum(self.stage_attention, outs, base=x)


class ProgressiveTSSA_Fusion(nn.Module):  # noqa: N801
    """Reference block.py:2632-2698."""

    def __init__(self, c, attn_ratio=0.5, num_heads=4, shortcut=True):
        super().__init__()
        self.c = c
        self.add = shortcut
        self.progressive_fusion1 = ProgressiveFeatureFusion(c, num_stages=3)
        self.progressive_fusion2 = ProgressiveFeatureFusion(c, num_stages=3)
        self.dyt1 = AdaptiveDynamicTanh(c, num_scales=3)
        self.dyt2 = AdaptiveDynamicTanh(c, num_scales=3)
        self.attn = CrossScaleAttentionTSSA(c, num_heads=num_heads, scales=[1, 2, 4])
        self.ffn = EDFFN(c, ffn_expansion_factor=2, bias=False)
        self.residual_weight1 = nn.Parameter(torch.tensor(0.1))
        self.residual_weight2 = nn.Parameter(torch.tensor(0.1))

    def forward(self, x):
        B, C, H, W = x.shape
        if self.add:
            identity, x = K.fanout(x)
        x = self.progressive_fusion1(x)
        a = K.untokens(self.attn(self.dyt1(x)), H, W)
        x = K.scale(a, self.residual_weight1, "scalar", res=identity) if self.add else a
        x = self.progressive_fusion2(x)
        if self.add:
            x, xr = K.fanout(x)
        f = self.ffn(self.dyt2(x))
        return K.scale(f, self.residual_weight2, "scalar", res=xr) if self.add else f


class Attention(nn.Module):
    """Multi-head self-attention over the H*W pixels (reference block.py:874-927): qkv 1x1 Conv+BN, per head
    q/k of key_dim = head_dim * attn_ratio and v of head_dim, softmax(q^T k * key_dim^-0.5), plus a depthwise
    3x3 positional encoding of v, then a 1x1 Conv+BN projection. The attention runs in the flash kernel
    (adr_attn_*, qk width 32, interleaved heads) straight on the NHWC qkv activation."""

    def __init__(self, dim, num_heads=8, attn_ratio=0.5):
        super().__init__()
        self.num_heads = num_heads
        self.head_dim = dim // num_heads
        self.key_dim = int(self.head_dim * attn_ratio)
        self.scale = self.key_dim ** -0.5
        nh_kd = self.key_dim * num_heads
        h = dim + nh_kd * 2
        self.qkv = Conv(dim, h, 1, act=False)
        self.proj = Conv(dim, dim, 1, act=False)
        self.pe = Conv(dim, dim, 3, 1, g=dim, act=False)

    def forward(self, x):
        o, v = K.psa_attention(self.qkv(x), self.num_heads, self.key_dim, self.head_dim)
        return self.proj(K.add(o, self.pe(v)))


class PSABlock(nn.Module):
    """Attention + FFN with shortcuts (reference block.py:930-967)."""

    def __init__(self, c, attn_ratio=0.5, num_heads=4, shortcut=True) -> None:
        super().__init__()
        self.attn = Attention(c, attn_ratio=attn_ratio, num_heads=num_heads)
        self.ffn = nn.Sequential(Conv(c, c * 2, 1), Conv(c * 2, c, 1, act=False))
        self.add = shortcut

    def forward(self, x):
        if not self.add:
            return self.ffn(self.attn(x))
        xa, xb = K.fanout(x)  # x feeds the residual and the branch: one HIP gradient sum
        x = K.add(xa, self.attn(xb))
        xa, xb = K.fanout(x)
        return K.add(xa, self.ffn(xb))


class C2PSA(nn.Module):
    """C2PSA (reference block.py:1010-1045): cv1 split, n PSABlocks on one half, concat, cv2. Subclasses
    (C2PTSSA, C2TSSA_DYT_Mona_EDFFN) replace self.m, as the reference's do."""

    def __init__(self, c1, c2, n=1, e=0.5):
        super().__init__()
        assert c1 == c2
        self.c = int(c1 * e)
        self.cv1 = Conv(c1, 2 * self.c, 1, 1)
        self.cv2 = Conv(2 * self.c, c1, 1)
        self.m = nn.Sequential(*(PSABlock(self.c, attn_ratio=0.5, num_heads=self.c // 64) for _ in range(n)))

    def forward(self, x, lazy=False):
        a, b = K.split(self.cv1(x), (self.c, self.c))
        b = self.m(b)
        return self.cv2(K.cat([a, b]), lazy=lazy)  # lazy: as C2f


class C2ProgressiveTSSA_Fusion(C2PSA):
    """Reference block.py:2700-2710 (alias C2PTSSA)."""

    def __init__(self, c1, c2, n=1, e=0.5):
        super().__init__(c1, c2, n, e)
        self.m = nn.Sequential(*(ProgressiveTSSA_Fusion(self.c, attn_ratio=0.5, num_heads=max(1, self.c // 64))
                                 for _ in range(n)))


C2PTSSA = C2ProgressiveTSSA_Fusion


# ------------------------------------------------------------------------------------------------------------
# 697 L10 variant: C2TSSA_DYT_Mona_EDFFN (reference block.py:1624-1709)
# ------------------------------------------------------------------------------------------------------------


class DynamicTanh(nn.Module):
    """Reference block.py:1624-1644: tanh(alpha x) * weight + bias (channels_first on this path)."""

    def __init__(self, normalized_shape, channels_last, alpha_init_value=0.5):
        super().__init__()
        if channels_last:
            raise NotImplementedError("the AD-Refine path uses DynamicTanh(channels_last=False) on NCHW maps")
        self.normalized_shape = normalized_shape
        self.alpha_init_value = alpha_init_value
        self.channels_last = channels_last
        self.alpha = nn.Parameter(torch.ones(1) * alpha_init_value)
        self.weight = nn.Parameter(torch.ones(normalized_shape))
        self.bias = nn.Parameter(torch.zeros(normalized_shape))

    def forward(self, x):
        return K.dyt(x, self.alpha, self.weight, self.bias)


class AttentionTSSA(nn.Module):
    """Reference block.py:1646-1683 over (B, C, N, 1) token tensors: qkv linear -> TSSA core -> to_out."""

    def __init__(self, dim, num_heads=8, qkv_bias=False, attn_drop=0.0, proj_drop=0.0, **kwargs):
        super().__init__()
        if attn_drop or proj_drop:
            raise NotImplementedError("AttentionTSSA dropout is 0 on the AD-Refine path")
        self.heads = num_heads
        self.qkv = nn.Linear(dim, dim, bias=qkv_bias)
        self.temp = nn.Parameter(torch.ones(num_heads, 1))
        self.to_out = nn.Sequential(nn.Linear(dim, dim), nn.Dropout(proj_drop))

    def forward(self, x_tok):
        w = _linear(x_tok, self.qkv.weight, self.qkv.bias)
        return _linear(K.tssa1(w, self.temp, self.heads), self.to_out[0].weight, self.to_out[0].bias)


class TSSAlock_DYT_Mona_EDFFN(nn.Module):  # noqa: N801 (reference name)
    """Reference block.py:1685-1703 (a PSABlock whose attn / ffn are replaced; attribute order as there, so the
    state_dict key order matches)."""

    def __init__(self, c, attn_ratio=0.5, num_heads=4, shortcut=True):
        super().__init__()
        self.attn = AttentionTSSA(c, num_heads=num_heads)
        self.ffn = EDFFN(c, ffn_expansion_factor=2, bias=False)
        self.add = shortcut
        self.dyt1 = DynamicTanh(normalized_shape=c, channels_last=False)
        self.dyt2 = DynamicTanh(normalized_shape=c, channels_last=False)
        self.mona1 = Mona(c)
        self.mona2 = Mona(c)

    def forward(self, x):
        B, C, H, W = x.shape
        a = K.untokens(self.attn(K.tokens(self.dyt1(x))), H, W)
        x = K.add(x, a) if self.add else a
        x = self.mona1(x)
        f = self.ffn(self.dyt2(x))
        x = K.add(x, f) if self.add else f
        return self.mona2(x)


class C2TSSA_DYT_Mona_EDFFN(C2PSA):  # noqa: N801
    """Reference block.py:1705-1709."""

    def __init__(self, c1, c2, n=1, e=0.5):
        super().__init__(c1, c2, n, e)
        self.m = nn.Sequential(*(TSSAlock_DYT_Mona_EDFFN(self.c, attn_ratio=0.5, num_heads=self.c // 64)
                                 for _ in range(n)))
