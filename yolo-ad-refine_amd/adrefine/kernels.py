"""Autograd wrappers over the libadr_hip C ABI.

Tensor convention: activations are logical NCHW tensors whose memory is NHWC (torch.channels_last), dtype
float32 (parity mode) or bfloat16 (performance mode). A channel slice of such a tensor is still an NHWC view
(pointer + per-pixel channel stride), so chunk/split/cat of channel groups cost nothing. Parameters stay
fp32 in the reference's own shapes (so state_dicts load unchanged) and are packed per step into the KRSC
operand layout in the compute dtype.

Every op here launches HIP kernels from libadr_hip.so; nothing falls back to PyTorch arithmetic.
"""
from __future__ import annotations

import ctypes

import torch

from .native import ConvDesc, lib

F32, BF16 = 0, 1
ACT = {"none": 0, "silu": 1, "gelu": 2, "relu": 3, "sigmoid": 4, "hswish": 5}
STATS_ROWS = 256  # rows per chunk for adr_nc_reduce

# counts layout fix-ups (should stay 0 on the hot path; tests assert it)
relayout_count = [0]


def dcode(dtype) -> int:
    if dtype == torch.float32:
        return F32
    if dtype == torch.bfloat16:
        return BF16
    raise RuntimeError(f"adrefine: unsupported activation dtype {dtype}")


def stream() -> int:
    return torch.cuda.current_stream().cuda_stream


def _req_cuda(t: torch.Tensor):
    if not t.is_cuda:
        raise RuntimeError("adrefine: HIP kernels need device tensors (no CPU fallback)")


def nhwc(t: torch.Tensor):
    """(tensor, ptr, cstride) for a logical NCHW tensor whose memory is an NHWC view; re-lays out otherwise."""
    _req_cuda(t)
    n, c, h, w = t.shape
    s0, s1, s2, s3 = t.stride()
    ok = (s1 == 1 or c == 1) and (s2 == w * s3 or h == 1) and (s0 == h * w * s3 or n == 1)
    vec = 16 // t.element_size()
    if not ok or t.data_ptr() % 16 or s3 % vec:
        relayout_count[0] += 1
        t = t.contiguous(memory_format=torch.channels_last)
        s3 = t.stride(3)
    return t, t.data_ptr(), s3


def empty_act(n, c, h, w, dtype, device):
    return torch.empty((n, h, w, c), dtype=dtype, device=device).permute(0, 3, 1, 2)


def fptr(t):
    return None if t is None else ctypes.c_void_p(t.data_ptr())


def pack_weight(w: torch.Tensor, dtype, cpad: int = 0, transpose_kc: int = 0):
    """(K, C, R, S) fp32 parameter -> KRSC operand in the compute dtype (channel-padded to cpad)."""
    K, C = w.shape[0], w.shape[1]
    RS = 1
    for d in w.shape[2:]:
        RS *= d
    Cp = max(C, cpad)
    out = torch.empty(K * RS * Cp, dtype=dtype, device=w.device)
    wf = w.detach()
    if wf.dtype != torch.float32 or not wf.is_contiguous():
        relayout_count[0] += 1
        wf = wf.float().contiguous()
    lib.adr_pack_weight(dcode(dtype), fptr(wf), fptr(out), K, C, Cp, RS, transpose_kc, stream())
    return out


def unpack_weight_grad(dw_krsc: torch.Tensor, shape, cpad: int = 0, transpose_kc: int = 0):
    K, C = shape[0], shape[1]
    RS = 1
    for d in shape[2:]:
        RS *= d
    out = torch.empty(shape, dtype=torch.float32, device=dw_krsc.device)
    lib.adr_unpack_weight_grad(fptr(dw_krsc), fptr(out), K, C, max(C, cpad), RS, transpose_kc, 0, stream())
    return out


def conv_desc(n, h, w, c, xcs, k, r, s, sh, sw, ph, pw, ycs, dtype):
    ho = (h + 2 * ph - r) // sh + 1
    wo = (w + 2 * pw - s) // sw + 1
    d = ConvDesc(n, h, w, c, xcs, 0, k, r, s, sh, sw, ph, pw, ho, wo, ycs, 0, dcode(dtype))
    return d, ho, wo


def _wgrad(d, xp, dyp, K, C, RS, device):
    dw = torch.empty(K * RS * C, dtype=torch.float32, device=device)
    ws_bytes = lib.adr_conv2d_wgrad_workspace(ctypes.byref(d))
    ws = torch.empty(max(ws_bytes // 4, 1), dtype=torch.float32, device=device)
    lib.adr_conv2d_wgrad(ctypes.byref(d), ctypes.c_void_p(xp), ctypes.c_void_p(dyp), fptr(dw), 0, fptr(ws),
                         ws_bytes, stream())
    return dw


def _bias_grad(dy, K, N, HW, cs):
    dt = dcode(dy.dtype)
    chunks = lib.adr_nc_reduce_chunks(HW, STATS_ROWS)
    part = torch.empty(N * chunks * 2 * K, dtype=torch.float32, device=dy.device)
    lib.adr_nc_reduce(dt, 0, ctypes.c_void_p(dy.data_ptr()), cs, 0, None, 0, 0, None, None, 0, 0, N, HW, K,
                      STATS_ROWS, fptr(part), stream())
    db = torch.empty(K, dtype=torch.float32, device=dy.device)
    lib.adr_partial_sum(fptr(part), N * chunks, K, 0, fptr(db), 0, stream())
    return db


class Conv2dFn(torch.autograd.Function):
    """y = conv2d(x, w) + b (dense, groups=1). Optionally also returns per-tile BN partial statistics."""

    @staticmethod
    def forward(ctx, x, w, b, stride, pad, want_stats, cpad):
        dtype = x.dtype
        x, xp, xcs = nhwc(x)
        N, C, H, W = x.shape
        K, Cw, R, S = w.shape
        Cp = max(Cw, cpad)
        if C != Cp:
            raise RuntimeError(f"Conv2dFn: input has {C} channels, weight expects {Cw} (padded {Cp})")
        wp = pack_weight(w, dtype, cpad)
        d, Ho, Wo = conv_desc(N, H, W, C, xcs, K, R, S, stride, stride, pad, pad, K, dtype)
        y = empty_act(N, K, Ho, Wo, dtype, x.device)
        stats = None
        if want_stats:
            tiles = lib.adr_conv2d_fwd_stat_tiles(ctypes.byref(d))
            stats = torch.empty(tiles * 2 * K, dtype=torch.float32, device=x.device)
        bf = b.detach().float().contiguous() if b is not None else None
        lib.adr_conv2d_fwd(ctypes.byref(d), ctypes.c_void_p(xp), fptr(wp), fptr(bf), ctypes.c_void_p(y.data_ptr()),
                           fptr(stats), 0, stream())
        ctx.save_for_backward(x, wp)
        ctx.meta = (stride, pad, cpad, w.shape, b is not None)
        if stats is None:
            stats = torch.empty(0, device=x.device)
        ctx.mark_non_differentiable(stats)
        return y, stats

    @staticmethod
    def backward(ctx, dy, _dstats):
        x, wp = ctx.saved_tensors
        stride, pad, cpad, wshape, has_b = ctx.meta
        dy, dyp, dycs = nhwc(dy.to(x.dtype) if dy.dtype != x.dtype else dy)
        N, C, H, W = x.shape
        K, _, R, S = wshape
        _, xp, xcs = nhwc(x)
        d, Ho, Wo = conv_desc(N, H, W, C, xcs, K, R, S, stride, stride, pad, pad, dycs, x.dtype)
        dx = dw = db = None
        if ctx.needs_input_grad[0]:
            dx = empty_act(N, C, H, W, x.dtype, x.device)
            d2, _, _ = conv_desc(N, H, W, C, C, K, R, S, stride, stride, pad, pad, dycs, x.dtype)
            lib.adr_conv2d_dgrad(ctypes.byref(d2), ctypes.c_void_p(dyp), fptr(wp), None,
                                 ctypes.c_void_p(dx.data_ptr()), 0, stream())
        if ctx.needs_input_grad[1]:
            dwk = _wgrad(d, xp, dyp, K, C, R * S, x.device)
            dw = unpack_weight_grad(dwk, wshape, cpad)
        if has_b and ctx.needs_input_grad[2]:
            db = _bias_grad(dy, K, N, Ho * Wo, dycs)
        return dx, dw, db, None, None, None, None


class ConvT2dFn(torch.autograd.Function):
    """nn.ConvTranspose2d(Cin, Cout, k, s, p, output_padding) forward = dgrad of the equivalent conv."""

    @staticmethod
    def forward(ctx, x, w, b, stride, pad, out_pad):
        dtype = x.dtype
        x, xp, xcs = nhwc(x)
        N, Ci, H, W = x.shape
        _, Co, R, S = w.shape
        Ho = (H - 1) * stride - 2 * pad + R + out_pad
        Wo = (W - 1) * stride - 2 * pad + S + out_pad
        wp = pack_weight(w, dtype)  # (Ci, Co, R, S) == KRSC of the equivalent conv (K=Ci, C=Co)
        y = empty_act(N, Co, Ho, Wo, dtype, x.device)
        d, h2, w2 = conv_desc(N, Ho, Wo, Co, Co, Ci, R, S, stride, stride, pad, pad, xcs, dtype)
        if (h2, w2) != (H, W):
            raise RuntimeError("ConvT2dFn: inconsistent geometry")
        bf = b.detach().float().contiguous() if b is not None else None
        lib.adr_conv2d_dgrad(ctypes.byref(d), ctypes.c_void_p(xp), fptr(wp), fptr(bf), ctypes.c_void_p(y.data_ptr()),
                             0, stream())
        ctx.save_for_backward(x, wp)
        ctx.meta = (stride, pad, w.shape, b is not None, Ho, Wo)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, wp = ctx.saved_tensors
        stride, pad, wshape, has_b, Ho, Wo = ctx.meta
        dy, dyp, dycs = nhwc(dy.to(x.dtype) if dy.dtype != x.dtype else dy)
        _, xp, xcs = nhwc(x)
        N, Ci, H, W = x.shape
        _, Co, R, S = wshape
        dx = dw = db = None
        if ctx.needs_input_grad[0]:
            dx = empty_act(N, Ci, H, W, x.dtype, x.device)
            d, _, _ = conv_desc(N, Ho, Wo, Co, dycs, Ci, R, S, stride, stride, pad, pad, Ci, x.dtype)
            lib.adr_conv2d_fwd(ctypes.byref(d), ctypes.c_void_p(dyp), fptr(wp), None, ctypes.c_void_p(dx.data_ptr()),
                               None, 0, stream())
        if ctx.needs_input_grad[1]:
            # equivalent conv: input = dy_T (N, Ho, Wo, Co), output grad = x_T (N, H, W, Ci)
            d, _, _ = conv_desc(N, Ho, Wo, Co, dycs, Ci, R, S, stride, stride, pad, pad, xcs, x.dtype)
            dwk = _wgrad(d, dyp, xp, Ci, Co, R * S, x.device)
            dw = unpack_weight_grad(dwk, wshape)
        if has_b and ctx.needs_input_grad[2]:
            db = _bias_grad(dy, Co, N, Ho * Wo, dycs)
        return dx, dw, db, None, None, None


class BNActFn(torch.autograd.Function):
    """act(BatchNorm2d(y)) — train mode uses batch statistics (from the conv epilogue when given)."""

    @staticmethod
    def forward(ctx, y, stats, gamma, beta, rm, rv, act, training, momentum, eps):
        dtype = y.dtype
        y, yp, ycs = nhwc(y)
        N, C, H, W = y.shape
        HW = H * W
        dev = y.device
        f = lambda: torch.empty(C, dtype=torch.float32, device=dev)  # noqa: E731
        scale, shift, mean, rstd = f(), f(), f(), f()
        if training:
            if stats is None or stats.numel() == 0:
                chunks = lib.adr_nc_reduce_chunks(HW, STATS_ROWS)
                stats = torch.empty(N * chunks * 2 * C, dtype=torch.float32, device=dev)
                lib.adr_nc_reduce(dcode(dtype), 0, ctypes.c_void_p(yp), ycs, 0, None, 0, 0, None, None, 0, 0, N, HW,
                                  C, STATS_ROWS, fptr(stats), stream())
            P = stats.numel() // (2 * C)
        else:
            P = 0
        lib.adr_bn_finalize(fptr(stats) if training else None, P, C, float(N * HW), fptr(gamma.detach()),
                            fptr(beta.detach()), fptr(rm), fptr(rv), float(momentum), float(eps), int(training),
                            fptr(scale), fptr(shift), fptr(mean), fptr(rstd), stream())
        z = empty_act(N, C, H, W, dtype, dev)
        lib.adr_affine_act(dcode(dtype), ctypes.c_void_p(yp), ycs, 0, ctypes.c_void_p(z.data_ptr()), C, 0,
                           fptr(scale), fptr(shift), 0, ACT[act], N, HW, C, stream())
        ctx.save_for_backward(y, scale, shift, mean, rstd, gamma)
        ctx.meta = (act, training)
        return z

    @staticmethod
    def backward(ctx, dz):
        y, scale, shift, mean, rstd, gamma = ctx.saved_tensors
        act, training = ctx.meta
        dz, dzp, dzcs = nhwc(dz.to(y.dtype) if dz.dtype != y.dtype else dz)
        _, yp, ycs = nhwc(y)
        N, C, H, W = y.shape
        HW = H * W
        dev = y.device
        dt = dcode(y.dtype)
        chunks = lib.adr_nc_reduce_chunks(HW, STATS_ROWS)
        part = torch.empty(N * chunks * 2 * C, dtype=torch.float32, device=dev)
        lib.adr_nc_reduce(dt, 1, ctypes.c_void_p(yp), ycs, 0, ctypes.c_void_p(dzp), dzcs, 0, fptr(scale), fptr(shift),
                          0, ACT[act], N, HW, C, STATS_ROWS, fptr(part), stream())
        f = lambda: torch.empty(C, dtype=torch.float32, device=dev)  # noqa: E731
        dgamma, dbeta, A, B, Cc = f(), f(), f(), f(), f()
        lib.adr_bn_bwd_finalize(fptr(part), N * chunks, C, float(N * HW), fptr(mean), fptr(rstd), fptr(gamma.detach()),
                                fptr(dgamma), fptr(dbeta), fptr(A), fptr(B), fptr(Cc), int(training), stream())
        dy = empty_act(N, C, H, W, y.dtype, dev)
        lib.adr_affine_act_bwd(dt, ctypes.c_void_p(yp), ycs, 0, ctypes.c_void_p(dzp), dzcs, 0,
                               ctypes.c_void_p(dy.data_ptr()), C, 0, fptr(scale), fptr(shift), fptr(A), fptr(B),
                               fptr(Cc), 0, 0, ACT[act], N, HW, C, 0, stream())
        return dy, None, dgamma, dbeta, None, None, None, None, None, None


class GNActFn(torch.autograd.Function):
    """act(GroupNorm(G)(y)) with per-(image, group) statistics."""

    @staticmethod
    def forward(ctx, y, gamma, beta, groups, act, eps):
        dtype = y.dtype
        y, yp, ycs = nhwc(y)
        N, C, H, W = y.shape
        HW = H * W
        dev = y.device
        chunks = lib.adr_nc_reduce_chunks(HW, STATS_ROWS)
        part = torch.empty(N * chunks * 2 * C, dtype=torch.float32, device=dev)
        lib.adr_nc_reduce(dcode(dtype), 0, ctypes.c_void_p(yp), ycs, 0, None, 0, 0, None, None, 0, 0, N, HW, C,
                          STATS_ROWS, fptr(part), stream())
        scale = torch.empty(N * C, dtype=torch.float32, device=dev)
        shift = torch.empty(N * C, dtype=torch.float32, device=dev)
        mean = torch.empty(N * groups, dtype=torch.float32, device=dev)
        rstd = torch.empty(N * groups, dtype=torch.float32, device=dev)
        lib.adr_gn_finalize(fptr(part), N, chunks, C, groups, float(HW * (C // groups)), fptr(gamma.detach()),
                            fptr(beta.detach()), float(eps), fptr(scale), fptr(shift), fptr(mean), fptr(rstd),
                            stream())
        z = empty_act(N, C, H, W, dtype, dev)
        lib.adr_affine_act(dcode(dtype), ctypes.c_void_p(yp), ycs, 0, ctypes.c_void_p(z.data_ptr()), C, 0,
                           fptr(scale), fptr(shift), 1, ACT[act], N, HW, C, stream())
        ctx.save_for_backward(y, scale, shift, mean, rstd, gamma)
        ctx.meta = (groups, act)
        return z

    @staticmethod
    def backward(ctx, dz):
        y, scale, shift, mean, rstd, gamma = ctx.saved_tensors
        groups, act = ctx.meta
        dz, dzp, dzcs = nhwc(dz.to(y.dtype) if dz.dtype != y.dtype else dz)
        _, yp, ycs = nhwc(y)
        N, C, H, W = y.shape
        HW = H * W
        dev = y.device
        dt = dcode(y.dtype)
        chunks = lib.adr_nc_reduce_chunks(HW, STATS_ROWS)
        part = torch.empty(N * chunks * 2 * C, dtype=torch.float32, device=dev)
        lib.adr_nc_reduce(dt, 1, ctypes.c_void_p(yp), ycs, 0, ctypes.c_void_p(dzp), dzcs, 0, fptr(scale), fptr(shift),
                          1, ACT[act], N, HW, C, STATS_ROWS, fptr(part), stream())
        dgamma = torch.empty(C, dtype=torch.float32, device=dev)
        dbeta = torch.empty(C, dtype=torch.float32, device=dev)
        A = torch.empty(N * C, dtype=torch.float32, device=dev)
        B = torch.empty(N * C, dtype=torch.float32, device=dev)
        Cc = torch.empty(N * C, dtype=torch.float32, device=dev)
        lib.adr_gn_bwd_finalize(fptr(part), N, chunks, C, groups, float(HW * (C // groups)), fptr(mean), fptr(rstd),
                                fptr(gamma.detach()), fptr(dgamma), fptr(dbeta), fptr(A), fptr(B), fptr(Cc), stream())
        dy = empty_act(N, C, H, W, y.dtype, dev)
        lib.adr_affine_act_bwd(dt, ctypes.c_void_p(yp), ycs, 0, ctypes.c_void_p(dzp), dzcs, 0,
                               ctypes.c_void_p(dy.data_ptr()), C, 0, fptr(scale), fptr(shift), fptr(A), fptr(B),
                               fptr(Cc), 1, 1, ACT[act], N, HW, C, 0, stream())
        return dy, dgamma, dbeta, None, None, None


def image_to_nhwc(img: torch.Tensor, dtype, cpad=8):
    """(B, 3, H, W) float images -> NHWC compute-dtype activation with channels padded to `cpad`."""
    _req_cuda(img)
    img = img.float()
    if not img.is_contiguous():
        relayout_count[0] += 1
        img = img.contiguous()
    N, C, H, W = img.shape
    out = empty_act(N, cpad, H, W, dtype, img.device)
    lib.adr_image_to_nhwc(dcode(dtype), fptr(img), ctypes.c_void_p(out.data_ptr()), N, C, H, W, cpad, stream())
    return out


# ---------------------------------------------------------------------------------------------------------
# functional entry points
# ---------------------------------------------------------------------------------------------------------


def conv2d(x, w, b=None, stride=1, pad=0, want_stats=False, cpad=0):
    y, stats = Conv2dFn.apply(x, w, b, stride, pad, want_stats, cpad)
    return y, stats


def conv_transpose2d(x, w, b, stride, pad, out_pad):
    return ConvT2dFn.apply(x, w, b, stride, pad, out_pad)


def bn_act(y, stats, bn: torch.nn.Module, act: str, training: bool):
    return BNActFn.apply(y, stats, bn.weight, bn.bias, bn.running_mean, bn.running_var, act, training, bn.momentum,
                         bn.eps)


def gn_act(y, gn: torch.nn.Module, act: str):
    return GNActFn.apply(y, gn.weight, gn.bias, gn.num_groups, act, gn.eps)
