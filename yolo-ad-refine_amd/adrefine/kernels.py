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
import weakref

import torch

from .native import ConvDesc, lib

F32, BF16 = 0, 1
ACT = {"none": 0, "silu": 1, "gelu": 2, "relu": 3, "sigmoid": 4, "hswish": 5}
_NC_MIN_BLOCKS = int(__import__("os").environ.get("ADR_NC_MIN_BLOCKS", 512))
# 1024 rows per chunk (was 256): fewer partial rows for the finalize kernels to walk; same-box sweep (4 runs each,
# scripts/ab_sweep.sh r06cb): 256 -> 19.54, 512 -> 19.50, 1024 -> 19.48 ms/step
_NC_ROWS = int(__import__("os").environ.get("ADR_NC_ROWS", 1024))


def _stats_rows(N, HW):
    """Rows per adr_nc_reduce chunk: 1024 (ADR_NC_ROWS), shrunk (in multiples of 32) on small maps until the
    reduction grid has ~_NC_MIN_BLOCKS workgroups — at 20x20 a 256-row chunk leaves 128 workgroups for the
    whole chip."""
    rows = _NC_ROWS
    if _NC_MIN_BLOCKS and N * -(-HW // rows) < _NC_MIN_BLOCKS:
        chunks = -(-_NC_MIN_BLOCKS // N)
        rows = max(32, -(-(-(-HW // chunks)) // 32) * 32)
    return rows


# counts layout fix-ups (should stay 0 on the hot path; tests assert it)
relayout_count = [0]
_TRACE_RELAYOUT = bool(int(__import__("os").environ.get("ADR_TRACE_RELAYOUT", "0")))


# ---------------------------------------------------------------------------------------------------------
# live per-kernel timing with HIP events on the launch stream (bench.py roofline); off unless timing_begin()
# ---------------------------------------------------------------------------------------------------------
_TIMING = None
_ANNOT = [0]  # > 0 inside an annotated _t0/_t1 region (its own bytes / flops; the generic hook stays out)


def timing_begin():
    """Time every libadr launch of the following eager work with HIP events on the launch stream: the conv / DCN
    paths annotate their launches with algorithmic bytes and flops (_t0/_t1); every other entry point is caught
    by the generic hook below, with bytes from _ALG_BYTES where the entry point has an estimator."""
    global _TIMING
    _TIMING = []
    from . import native
    native.CALL_HOOK = _hook_call


def timing_end():
    global _TIMING
    global _DETAIL
    from . import native
    native.CALL_HOOK = None
    recs, _TIMING = _TIMING, None
    if not recs:
        return []
    torch.cuda.synchronize()
    _DETAIL = [(tag, shape, nb, fl, e0.elapsed_time(e1) * 1e-3 / rep) for tag, nb, fl, e0, e1, shape, rep in recs]
    return [(tag, nbytes, flops, e0.elapsed_time(e1) * 1e-3 / rep) for tag, nbytes, flops, e0, e1, _, rep in recs]


def timing_detail():
    """After timing_end(): per-launch (tag, shape, bytes, flops, seconds) of the last timed region."""
    return _DETAIL


_DETAIL = []


# Timed launches that are idempotent (they overwrite their outputs) run TIMING_REPEAT times back to back between
# the two events, so the per-launch dispatch gap the events also bracket is amortised: the per-launch figure then
# matches the kernel's own duration (rocprofv3 --kernel-trace) instead of exceeding it by the gap.
TIMING_REPEAT = 4


def _reps(accumulate=0):
    return TIMING_REPEAT if _TIMING is not None and not accumulate else 1


def _t0(tag, nbytes, flops, shape="", rep=1):
    if _TIMING is None:
        return None
    _ANNOT[0] += 1
    e0 = torch.cuda.Event(enable_timing=True)
    e0.record()
    return (tag, nbytes, flops, e0, shape, rep)


def _t1(tok):
    if tok is not None:
        _ANNOT[0] -= 1
        e1 = torch.cuda.Event(enable_timing=True)
        e1.record()
        tag, nb, fl, e0, shape, rep = tok
        _TIMING.append((tag, nb, fl, e0, e1, shape, rep))


def _es(dtype_code):
    return 2 if dtype_code == BF16 else 4


# entry point -> (kernel label as rocprofv3 names it, algorithmic bytes from the call's arguments, idempotent?)
# Algorithmic bytes: every tensor the launch must touch, read or written once (NHWC activations, compute dtype).
_ALG_BYTES = {
    "adr_affine_act_bwd": (lambda a: f"adr::affine_act_bwd_kernel<__bf16, {a[17]}>",
                           lambda a: _es(a[0]) * a[18] * a[19] * a[20] * (3 + a[21]), lambda a: a[21] == 0),
    "adr_affine_act": (lambda a: f"adr::affine_act_kernel<__bf16, {a[10]}>",
                       lambda a: _es(a[0]) * a[11] * a[12] * a[13] * 2, lambda a: True),
    "adr_nc_reduce": (lambda a: f"adr::nc_reduce_kernel<__bf16, {1 if a[1] == 1 else 0}, {a[11] if a[1] == 1 else 0}>",
                      lambda a: _es(a[0]) * a[12] * a[13] * a[14] * (2 if a[1] == 1 else 1), lambda a: True),
    "adr_ew": ("adr::ew_kernel<__bf16>",
               lambda a: _es(a[0]) * a[11] * a[12] * (2 + (a[5] is not None) + (a[7] is not None) + a[15]),
               lambda a: a[15] == 0 and _ptr(a[9]) not in (_ptr(a[3]), _ptr(a[5]), _ptr(a[7]))),
}


def _ptr(v):
    return v.value if isinstance(v, ctypes.c_void_p) else v


def _entries(args, struct):
    """The ctypes entry array a batched entry point was handed (args[0] = pointer, args[1] = count)."""
    n = int(args[1])
    return ctypes.cast(args[0], ctypes.POINTER(struct))[:n] if n > 0 and _ptr(args[0]) else []


# batched entry points: algorithmic bytes summed over their entries (each entry's tensors touched once)
_BATCHED_BYTES = {
    "adr_wgrad_reduce_batched": lambda a: sum(
        4 * (e.splits * e.K * e.RS * e.Cp + e.K * e.C * e.RS * (2 if e.accumulate else 1))
        for e in _entries(a, WgradEntry)),
    "adr_nc_reduce_batched": lambda a: sum(2 * e.N * e.HW * e.C + 4 * e.N * e.chunks * 2 * e.C
                                           for e in _entries(a, ColsumEntry)),
    "adr_partial_sum_batched": lambda a: sum(4 * (e.P * e.C + e.C * (2 if e.accumulate else 1))
                                             for e in _entries(a, PsumEntry)),
    "adr_axpy_batched": lambda a: sum(12 * e.n for e in _entries(a, AxpyEntry)),
    "adr_gn_param_grad_batched": lambda a: sum(
        4 * (e.N * e.chunks * 2 * e.C + 2 * e.N * e.G + 2 * e.C * (2 if e.accumulate else 1))
        for e in _entries(a, GnParamEntry)),
    "adr_dotsum_batched": lambda a: sum(4 * e.N * e.HW * e.C + 4 * e.N * e.chunks * 2 * e.C
                                        for e in _entries(a, DotsumEntry)),
    "adr_copy_pieces": lambda a: sum(4 * int(a[2]) * e.C for e in _entries(a, CopyPiece)),
    # fp32 weights read once, both bf16 layouts written (PackCache._build records the sum per table)
    "adr_pack_weight2_tiled": lambda a: _PACK_BYTES.get(_ptr(a[1]), 0),
}
_PACK_BYTES = {}  # device table pointer -> algorithmic bytes of one adr_pack_weight2_tiled launch


def _scan_tensors(v, want, found, depth=0):
    if torch.is_tensor(v):
        if v.is_cuda:
            p = v.data_ptr()
            if p in want:
                found[p] = max(found.get(p, 0), v.numel() * v.element_size())
        return
    if depth < 1 and isinstance(v, (tuple, list)) and len(v) <= 64:
        for u in v:
            _scan_tensors(u, want, found, depth + 1)


def _generic_bytes(name, args):
    """Algorithmic bytes of an entry point without its own estimator: the logical size of every device tensor it is
    handed (each read or written once), found by matching its pointer arguments against the tensors live in the
    calling frames (the autograd Function that issued it). None when no pointer matched."""
    import sys
    types_ = lib.protos.get(name, (None, []))[1]
    want = {_ptr(a) for a, t in zip(args, types_) if t is ctypes.c_void_p and _ptr(a)}
    if not want:
        return None
    found = {}
    f = sys._getframe(3)
    for _ in range(4):
        if f is None or len(found) == len(want):
            break
        for v in list(f.f_locals.values()):
            _scan_tensors(v, want, found)
        f = f.f_back
    return sum(found.values()) if found else None


_UNTIMED = ("_symbol", "_workspace", "_splits", "_tiles", "_chunks", "_size", "_floats", "_supported", "adr_set_f32")


_SITE_LABELS = ("adr_ew", "adr_affine_act", "adr_affine_act_bwd", "adr_nc_reduce", "adr_memset_zero",
                "adr_bcast_mul", "adr_cast")


def _call_site():
    """The first caller outside this module's launch helpers (timing detail labels: which op issued a launch)."""
    import sys
    f = sys._getframe(2)
    while f is not None and f.f_code.co_name in ("_ew", "_hook_call", "wrapper", "call", "__call__", "_call"):
        f = f.f_back
    if f is None:
        return "?"
    cls = f.f_locals.get("ctx")
    owner = type(cls).__name__.replace("Backward", "") if cls is not None else ""
    return f"{owner}.{f.f_code.co_name}:{f.f_lineno}" if owner else f"{f.f_code.co_name}:{f.f_lineno}"


# algorithmic flops of the generic entry points that run matrix work (the rest are byte-bound: 0)
# flash attention: forward S = Q K^T and O = P V; backward the standard five products (S recomputed, dV = P^T dO,
# dP = dO V^T, dQ = dS K, dK = dS^T Q) — 2 B h L^2 per unit of width (q/k width dqk, v width dv)
_ALG_FLOPS = {
    "adr_attn_fwd": lambda a: 2.0 * a[11] * a[13] * a[12] ** 2 * (a[14] + a[15]),
    "adr_attn_bwd": lambda a: 2.0 * a[21] * a[23] * a[22] ** 2 * (3 * a[24] + 2 * a[25]),
}


def _hook_call(name, fn, args):
    """Generic timing of one libadr call (outside annotated regions; host-side queries are not timed)."""
    if _TIMING is None or _ANNOT[0] > 0 or name.endswith(_UNTIMED):
        rc = fn(*args)
    else:
        spec = _ALG_BYTES.get(name)
        label, nbytes, rep = name, None, 1
        if spec is not None:
            label = spec[0](args) if callable(spec[0]) else spec[0]
            if args[0] != BF16:
                label = label.replace("__bf16", "float")
            nbytes = int(spec[1](args))
            rep = TIMING_REPEAT if spec[2](args) else 1
        elif name in _BATCHED_BYTES:
            nbytes = int(_BATCHED_BYTES[name](args))
        else:
            nbytes = _generic_bytes(name, args)
        flops = int(_ALG_FLOPS[name](args)) if name in _ALG_FLOPS else 0
        shape = _call_site() if name in _SITE_LABELS else ""
        if name == "adr_ew":
            shape = f"op{args[1]}{'+acc' if args[15] else ''} {args[11]}px x{args[12]}ch @{shape}"
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        rc = 0
        for _ in range(rep):
            rc = fn(*args)
            if rc != 0:
                break
        e1.record()
        _TIMING.append((label, nbytes, flops, e0, e1, shape, rep))
    if rc != 0:
        raise RuntimeError(f"{name}: {lib.lib.adr_last_error().decode()}")
    return rc


def _bn_of(n):
    return 16 if n <= 16 else 32 if n <= 32 else 64 if n <= 64 else 128


def roofline_report(recs, dtype, hbm_gbs, mfma_tf):
    """The dominant kernel of the measured step (largest total time over every timed launch) -> achieved
    algorithmic GB/s or TF/s against the bound that applies to it (HBM below the ridge, MFMA above)."""
    if not recs:
        return None
    agg = {}
    for tag, nb, fl, t in recs:
        a = agg.setdefault(tag, [0, 0.0, 0.0, 0.0, True])
        a[0] += 1
        a[1] += nb or 0
        a[2] += fl or 0
        a[3] += t
        a[4] = a[4] and nb is not None
    total_t = sum(v[3] for v in agg.values())
    # whole-step accounting: per label, ideal = max(bytes / HBM peak, flops / MFMA peak) summed over its launches;
    # lost = measured - ideal; worst = the label losing the most time (labels without bytes count as all lost)
    ideal = {}
    for tag_, nb_, fl_, t_ in recs:
        ideal[tag_] = ideal.get(tag_, 0.0) + max((nb_ or 0) / (hbm_gbs * 1e9), (fl_ or 0) / (mfma_tf * 1e12))
    known_t = sum(v[3] for v in agg.values() if v[4])
    known_ideal = sum(ideal[k] for k, v in agg.items() if v[4])
    lost = {k: v[3] - ideal[k] for k, v in agg.items()}
    wk = max(lost, key=lost.get)
    worst = {"kernel": wk, "launches": agg[wk][0], "ms_total": round(1e3 * agg[wk][3], 3),
             "lost_ms": round(1e3 * lost[wk], 3), "attainable_frac": round(ideal[wk] / agg[wk][3], 4)
             if agg[wk][4] else None, "has_bytes": agg[wk][4]}
    step = {"timed_ms": round(1e3 * total_t, 3), "launches": sum(v[0] for v in agg.values()),
            "ms_with_alg_bytes": round(1e3 * known_t, 3), "ms_without_alg_bytes": round(1e3 * (total_t - known_t), 3),
            "labels_without_alg_bytes": sorted(k for k, v in agg.items() if not v[4]),
            "ideal_ms": round(1e3 * known_ideal, 3),
            "attainable_frac": round(known_ideal / known_t, 4) if known_t else None,
            "alg_bytes": int(sum(v[1] for v in agg.values())), "alg_flops": int(sum(v[2] for v in agg.values()))}
    tag, (cnt, nb, fl, t, known) = max(agg.items(), key=lambda kv: kv[1][3])
    gbs = nb / t / 1e9 if known else None
    tfs = fl / t / 1e12
    ridge = mfma_tf * 1e12 / (hbm_gbs * 1e9)
    ai = fl / max(nb, 1)
    bound = "mfma" if ai > ridge else "hbm"
    achieved, peak, unit = (tfs, mfma_tf, "TFLOP/s") if bound == "mfma" else (gbs, hbm_gbs, "GB/s")
    return {"bound": bound, "achieved": None if achieved is None else round(achieved, 2), "peak": peak, "unit": unit,
            "frac": None if achieved is None else round(achieved / peak, 4), "traffic": None, "kernel": tag,
            "launches": cnt, "avg_us": round(1e6 * t / cnt, 2), "alg_bytes_per_launch": int(nb / cnt),
            "alg_flops_per_launch": int(fl / cnt), "achieved_gbs": None if gbs is None else round(gbs, 1),
            "achieved_tfs": round(tfs, 2), "share_of_timed_time": round(t / total_t, 3),
            "worst": worst, "step": step,
            "kernels": {k: {"launches": v[0], "ms_total": round(1e3 * v[3], 3), "avg_us": round(1e6 * v[3] / v[0], 2),
                            "gbs": round(v[1] / v[3] / 1e9, 1) if v[4] and v[1] else None,
                            "tfs": round(v[2] / v[3] / 1e12, 2) if v[2] else None,
                            "frac": round(ideal[k] / v[3], 4) if v[4] else None}
                        for k, v in sorted(agg.items(), key=lambda kv: -kv[1][3])[:40]}}


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
    """(tensor, ptr, cstride) for a logical NCHW tensor whose memory is an NHWC view; re-lays out otherwise. A
    BN-act output still pending for its consumer conv (BnFwd) is written first when anything else reads it."""
    _req_cuda(t)
    if _BNF_PENDING:
        _bnf_settle(t)
    n, c, h, w = t.shape
    s0, s1, s2, s3 = t.stride()
    ok = (s1 == 1 or c == 1) and (s2 == w * s3 or h == 1) and (s0 == h * w * s3 or n == 1)
    vec = 16 // t.element_size()
    if not ok or t.data_ptr() % 16 or s3 % vec:
        relayout_count[0] += 1
        if _TRACE_RELAYOUT:
            import traceback
            traceback.print_stack(limit=6)
        t = t.contiguous(memory_format=torch.channels_last)
        s3 = t.stride(3)
    return t, t.data_ptr(), s3


def empty_act(n, c, h, w, dtype, device):
    return torch.empty((n, h, w, c), dtype=dtype, device=device).permute(0, 3, 1, 2)


def fptr(t):
    return None if t is None else ctypes.c_void_p(t.data_ptr())


def _target(t):
    """The Parameter owning gradient-arena storage for t (t itself, or the base of a reshaped view)."""
    if t is None:
        return None
    if hasattr(t, "_adr_grad"):
        return t
    b = getattr(t, "_base", None)
    if b is not None and hasattr(b, "_adr_grad"):
        return b
    return None


def sink(t, g):
    """Route a parameter gradient: accumulate into the trainer's flat fp32 gradient arena when the parameter
    has one (returns None to autograd), otherwise hand it back to autograd unchanged."""
    if g is None:
        return None
    tgt = _target(t)
    if tgt is None:
        return g
    gc = g.detach().float()
    if not gc.is_contiguous():
        relayout_count[0] += 1
        gc = gc.contiguous()
    if gc.numel() != tgt.numel():
        raise RuntimeError("sink: gradient size mismatch")
    dst = _grad_buf(tgt)
    if _dfr() is not None and _TIMING is None:
        _dfr().add_axpy(gc, dst.data_ptr(), gc.numel())
    else:
        lib.adr_axpy(gc.numel(), 1.0, fptr(gc), fptr(dst), stream())
    tgt._adr_used = True
    return None


def grad_dst(t, numel, device):
    """Where a kernel should write the gradient of parameter t: (tensor-or-None, ptr, accumulate). With a trainer
    arena the kernel accumulates straight into t's arena slice (no temporary, no axpy launch) and autograd gets
    None; otherwise a fresh fp32 buffer is returned for autograd."""
    tgt = _target(t)
    if tgt is not None:
        if tgt.numel() != numel:
            raise RuntimeError("grad_dst: gradient size mismatch")
        tgt._adr_used = True
        return None, fptr(_grad_buf(tgt)), 1
    out = torch.empty(numel, dtype=torch.float32, device=device)
    return out, fptr(out), 0


def grad_ret(t, buf):
    """The autograd return value for a grad_dst destination (reshaped to the parameter)."""
    return None if buf is None else buf.view(t.shape)


def sink_unpack(t, dw_krsc, shape, cpad=0):
    """unpack_weight_grad straight into the gradient arena (accumulate) when t has one."""
    tgt = _target(t)
    if tgt is None:
        return unpack_weight_grad(dw_krsc, shape, cpad)
    K_, C_ = shape[0], shape[1]
    RS = 1
    for d in shape[2:]:
        RS *= d
    lib.adr_unpack_weight_grad(fptr(dw_krsc), fptr(_grad_buf(tgt)), K_, C_, max(C_, cpad), RS, 0, 1, stream())
    tgt._adr_used = True
    return None


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


def _pair(v):
    return (v, v) if isinstance(v, int) else (int(v[0]), int(v[1]))


def conv_desc(n, h, w, c, xcs, k, r, s, sh, sw, ph, pw, ycs, dtype):
    ho = (h + 2 * ph - r) // sh + 1
    wo = (w + 2 * pw - s) // sw + 1
    d = ConvDesc(n, h, w, c, xcs, 0, k, r, s, sh, sw, ph, pw, ho, wo, ycs, 0, dcode(dtype))
    return d, ho, wo


def _gemm_symbol(dtype_code, bn, mode):
    """Kernel symbol of adr_gemm.hip's gemm_kernel<T, BN, MODE> as rocprofv3 reports it."""
    t = "DF16b" if dtype_code == BF16 else "f"
    return f"_ZN3adr11gemm_kernelI{t}Li{bn}ELi{mode}EEEvNS_8GemmArgsE"


def _shape(d, mode):
    return (f"{mode} n{d.n} {d.h}x{d.w} c{d.c}/{d.x_cstride} -> k{d.k}/{d.y_cstride} {d.r}x{d.s} "
            f"s{d.stride_h} o{d.ho}x{d.wo}")


def _conv_work(d):
    """(algorithmic bytes, flops) of one dense conv contraction: x, w, y each touched once."""
    es = 2 if d.dtype == BF16 else 4
    nbytes = es * (d.n * d.h * d.w * d.c + d.k * d.r * d.s * d.c + d.n * d.ho * d.wo * d.k)
    return nbytes, 2 * d.n * d.ho * d.wo * d.k * d.r * d.s * d.c


def _engine2(d, red_channels):
    """Every bf16 contraction runs on the BK-64 engine (adr_conv.hip); with its division-free tap decoder it
    measures faster than the generic engine on every shape of the step (scripts/conv_s1.sh, conv_shapes.sh),
    including the ELA 7x1 Conv1d (padding (3, 0)): 33-65 us per launch on the generic engine."""
    return d.dtype == BF16 and d.stride_h == d.stride_w


def _conv2_symbol(d, dgrad):
    """The bf16 engine's kernel for this contraction, as the library dispatches it (roofline label)."""
    buf = ctypes.create_string_buffer(128)
    lib.adr_conv2d_bf16_kernel_symbol(ctypes.byref(d), int(dgrad), buf, 128)
    return buf.value.decode()


def conv_fwd(d, xp, wp, bias, yp, stats=None, accumulate=0):
    """y (+)= conv(x, w_krsc) (+bias); optional per-128-row-tile BN partial statistics of the stored values."""
    e2 = _engine2(d, d.c)
    sym = "" if _TIMING is None else _conv2_symbol(d, False) if e2 else _gemm_symbol(d.dtype, _bn_of(d.k), 0)
    rep = _reps(accumulate)
    tok = _t0(sym, *_conv_work(d), _shape(d, "fwd") if _TIMING is not None else "", rep)
    fn = lib.adr_conv2d_fwd_bf16 if e2 else lib.adr_conv2d_fwd
    for _ in range(rep):
        fn(ctypes.byref(d), ctypes.c_void_p(xp), ctypes.c_void_p(wp), bias, ctypes.c_void_p(yp), stats,
           int(accumulate), stream())
    _t1(tok)


# BASELINE.json configs[4]'s fp8 MFMA conv path: bias-free forward convs (Conv-BN-act) with a spatial kernel and
# >= _FP8_MIN_C input channels run on the e4m3 engine (adr_conv_fp8.hip) when set (bench.py --conv-fp8, or
# ADR_CONV_FP8=1); backward stays bf16. Measured (scripts/fp8_micro.py, l-scale 1280^2 bs16 shapes): 3x3 convs
# with C >= 128 run 1.04-1.24x faster than on the bf16 engine; 1x1 and 64-channel convs are memory-bound and
# gain nothing (the staging conversion costs VALU), so they stay bf16.
CONV_FP8 = bool(int(__import__("os").environ.get("ADR_CONV_FP8", "0")))
_FP8_MIN_C = 128


def conv_fwd_fp8(d, xp, w, Cw, Cp, bias, yp, stats):
    """y = conv(x, w) (+bias) on the fp8 engine with delayed per-tensor activation scaling: the conv collects its
    input's |x| maxima for the next step as it stages x; the per-step weight pack (per output channel) rotates
    them (state on the weight tensor: [amax_cur, amax_prev]). The first call seeds the maxima with one
    adr_amax_bf16 pass over x."""
    dev = w.device
    K_, RS = w.shape[0], w.shape[2] * w.shape[3]
    nb = lib.adr_fp8_amax_blocks()
    st = getattr(w, "_adr_fp8", None)
    if st is None:
        st = [torch.zeros(nb, dtype=torch.float32, device=dev), torch.zeros(nb, dtype=torch.float32, device=dev)]
        w._adr_fp8 = st
        lib.adr_amax_bf16(ctypes.c_void_p(xp), d.x_cstride, 0, d.n * d.h * d.w, d.c, fptr(st[0]), stream())
    w8 = torch.empty(K_ * RS * Cp, dtype=torch.uint8, device=dev)
    winv = torch.empty(K_, dtype=torch.float32, device=dev)
    lib.adr_pack_weight_fp8(fptr(w.detach().float().contiguous()), K_, Cw, Cp, RS, fptr(w8), fptr(winv), fptr(st[0]),
                            fptr(st[1]), stream())
    lib.adr_conv2d_fwd_fp8(ctypes.byref(d), ctypes.c_void_p(xp), fptr(w8), fptr(winv), fptr(st[1]), fptr(st[0]),
                           fptr(bias), ctypes.c_void_p(yp), fptr(stats), stream())


def conv_dgrad(d, dyp, wpair, bias, dxp, accumulate=0, addend=None, xf=None, dy=None, bst=None, dx=None):
    """dx (+)= conv_transpose(dy, w) (+ addend); wpair = (KRSC, CRSK-or-None) packed weights (pack_weight2).
    `addend` (an NHWC bf16 view shaped like dx) is added in the bf16 engine's epilogue. With `xf` (a BnXf) the
    operand is the BN-act backward of xf.dz, applied while staging and side-written into `dy` (which dyp is not
    read from). With `bst` (a BnStat: dx is the complete dz of that BN) the epilogue also writes the BN's backward
    statistics partials (BSTAT), handed to the BnStat for its BNActFn.backward."""
    krsc, crsk = wpair
    e2 = crsk is not None and _engine2(d, d.k)
    mode = 2 if d.stride_h == 2 else 1
    if bst is not None:
        st = None
        if xf is not None:
            _, dzp, dzcs = nhwc(xf.dz)
            d.y_cstride = dzcs
            dyp = dzp
            st = xf.struct(dy)
        P = lib.adr_conv2d_dgrad_bf16_stat_tiles(ctypes.byref(d), int(xf is not None))
        part = torch.empty(P * 2 * d.c, dtype=torch.float32, device=dx.device)
        bs = bst.struct()
        sym = "" if _TIMING is None else _conv2_symbol(d, 5 | (2 if xf is not None else 0))
        tok = _t0(sym, *_conv_work(d), _shape(d, "dgrad+bstat" + ("+bnact" if xf is not None else ""))
                  if _TIMING is not None else "")
        lib.adr_conv2d_dgrad_bf16_bstat(ctypes.byref(d), ctypes.c_void_p(dyp), ctypes.c_void_p(crsk.data_ptr()),
                                        ctypes.c_void_p(dxp), int(accumulate),
                                        None if addend is None else ctypes.c_void_p(addend.data_ptr()),
                                        0 if addend is None else addend.stride(3),
                                        None if st is None else ctypes.byref(st), ctypes.byref(bs), fptr(part),
                                        stream())
        _t1(tok)
        bst.set(part, P, dx)
        return
    if xf is not None:
        _, dzp, dzcs = nhwc(xf.dz)
        d.y_cstride = dzcs  # the operand's view: dz (dy shares its pixel grid, written through the side output)
        st = xf.struct(dy)
        sym = "" if _TIMING is None else _conv2_symbol(d, 3)
        tok = _t0(sym, *_conv_work(d), _shape(d, "dgrad+bnact") if _TIMING is not None else "")
        lib.adr_conv2d_dgrad_bf16_bnact(ctypes.byref(d), ctypes.c_void_p(dzp), ctypes.c_void_p(crsk.data_ptr()),
                                        ctypes.c_void_p(dxp), int(accumulate),
                                        None if addend is None else ctypes.c_void_p(addend.data_ptr()),
                                        0 if addend is None else addend.stride(3), ctypes.byref(st), stream())
        _t1(tok)
        return
    sym = "" if _TIMING is None else (_conv2_symbol(d, True) if e2 else
                                      _gemm_symbol(d.dtype, _bn_of(d.c), 3 if mode == 2 else 1))
    if addend is not None:
        if not e2 or bias is not None:
            raise RuntimeError("conv_dgrad: an addend needs the bf16 engine and no bias")
        tok = _t0(sym, *_conv_work(d), _shape(d, "dgrad+add") if _TIMING is not None else "")
        lib.adr_conv2d_dgrad_bf16_add(ctypes.byref(d), ctypes.c_void_p(dyp), ctypes.c_void_p(crsk.data_ptr()),
                                      ctypes.c_void_p(dxp), int(accumulate), ctypes.c_void_p(addend.data_ptr()),
                                      addend.stride(3), stream())
        _t1(tok)
        return
    rep = _reps(accumulate)
    tok = _t0(sym, *_conv_work(d), _shape(d, "dgrad") if _TIMING is not None else "", rep)
    for _ in range(rep):
        if e2:
            lib.adr_conv2d_dgrad_bf16(ctypes.byref(d), ctypes.c_void_p(dyp), ctypes.c_void_p(crsk.data_ptr()), bias,
                                      ctypes.c_void_p(dxp), int(accumulate), stream())
        else:
            lib.adr_conv2d_dgrad(ctypes.byref(d), ctypes.c_void_p(dyp), ctypes.c_void_p(krsc.data_ptr()), bias,
                                 ctypes.c_void_p(dxp), int(accumulate), stream())
    _t1(tok)


class PackCache:
    """Per-trainer cache of the bf16 conv operand copies (KRSC + CRSK) of every conv weight. The first step
    records each (weight, layout) pair and packs it into a persistent buffer; from then on `pack_all()` repacks
    all of them in ONE batched launch at the start of the step (inside the captured graph), and pack_weight2
    returns the cached buffers until the optimizer invalidates them."""

    def __init__(self, cache_bn_coefs=False):
        self.specs = {}
        self.valid = False
        self.table = None
        self.nchunks = 0
        self.tab_dev = None
        # eval Conv-BN-act: the running-statistics scale/shift per BatchNorm, computed once and refreshed by
        # refresh_bn_coefs() (the predictor's sync_weights) — only where the owner guarantees fixed weights
        self.cache_bn_coefs = cache_bn_coefs
        self.bn_coefs = {}

    def refresh_bn_coefs(self):
        for bn, scale, shift in self.bn_coefs.values():
            _bn_eval_coefs_into(bn, scale, shift)

    def _build(self):
        """One row per (weight, tap, 64 x 64 tile) for adr_pack_weight2_tiled (coalesced stores in both layouts)."""
        import numpy as np
        dt = np.dtype([("src", "<u8"), ("krsc", "<u8"), ("crsk", "<u8"), ("K", "<i4"), ("Kp", "<i4"), ("C", "<i4"),
                       ("Cp", "<i4"), ("RS", "<i4"), ("tkc", "<i4"), ("t", "<i4"), ("k0", "<i4"), ("c0", "<i4"),
                       ("pad", "<i4")])
        assert dt.itemsize == lib.adr_pack_tile_size()
        rows = []
        for sp in self.specs.values():
            w, K, Kp, C, Cp, RS, tkc, krsc, crsk = sp
            for t in range(RS):
                for k0 in range(0, Kp, 64):
                    for c0 in range(0, Cp, 64):
                        rows.append((w.data_ptr(), krsc.data_ptr(), crsk.data_ptr(), K, Kp, C, Cp, RS, tkc, t, k0,
                                     c0, 0))
        tab = np.array(rows, dtype=dt)
        dev = next(iter(self.specs.values()))[0].device
        self.tab_dev = torch.from_numpy(tab.view(np.uint8).copy()).to(dev)
        _PACK_BYTES[self.tab_dev.data_ptr()] = sum(4 * K * C * RS + 2 * 2 * Kp * Cp * RS
                                                   for _, K, Kp, C, Cp, RS, _, _, _ in self.specs.values())
        self.nchunks = len(rows)
        self.table = len(self.specs)

    def pack_all(self):
        if not self.specs:
            return
        if self.table != len(self.specs):
            self._build()
        lib.adr_pack_weight2_tiled(BF16, fptr(self.tab_dev), self.nchunks, stream())
        self.valid = True


_PACK = None  # the active PackCache (set by the trainer around its forward/backward)


def pack_scope(cache):
    """Context manager activating a PackCache."""
    import contextlib

    @contextlib.contextmanager
    def _cm():
        global _PACK
        prev, _PACK = _PACK, cache
        try:
            yield cache
        finally:
            _PACK = prev
    return _cm()


def pack_weight2(w: torch.Tensor, dtype, cpad: int = 0, transpose_kc: int = 0, kpad: int = 0):
    """(K, C, R, S) fp32 parameter -> (KRSC [Kp][RS][Cp], CRSK [Cp][RS][Kp]) operands in one launch for bf16
    (the CRSK copy feeds the bf16 data-gradient engine); (KRSC, None) for fp32. Under an active PackCache the
    operands come from (or are recorded into) its persistent buffers."""
    pc = _PACK
    # a reshaped view of a parameter (nn.Linear / Conv1d weights used as 1x1 / 7x1 conv weights) is a new tensor
    # on every call: it is keyed by its storage and geometry instead, so it is packed once too
    view = isinstance(w._base, torch.nn.Parameter)  # (a leaf under no_grad, but still a new object per call)
    key = ((w.data_ptr(), tuple(w.shape), tuple(w.stride())) if view else id(w), cpad, transpose_kc, kpad)
    if pc is not None and dtype == torch.bfloat16 and pc.valid and key in pc.specs:
        sp = pc.specs[key]
        return sp[7], sp[8]
    if dtype != torch.bfloat16:
        if kpad and kpad != w.shape[0]:
            raise RuntimeError("pack_weight2: output-channel padding is bf16-only")
        return pack_weight(w, dtype, cpad, transpose_kc), None
    if transpose_kc:
        C, K = w.shape[0], w.shape[1]
    else:
        K, C = w.shape[0], w.shape[1]
    RS = 1
    for v in w.shape[2:]:
        RS *= v
    Cp, Kp = max(C, cpad), max(K, kpad)
    wf = w.detach()
    direct = wf.dtype == torch.float32 and wf.is_contiguous()
    if not direct:
        relayout_count[0] += 1
        wf = wf.float().contiguous()
    if pc is not None and direct and (w.is_leaf or view):  # record: persistent buffers, repacked by pack_all
        sp = pc.specs.get(key)
        if sp is None:
            sp = (w, K, Kp, C, Cp, RS, transpose_kc, torch.empty(Kp * RS * Cp, dtype=dtype, device=w.device),
                  torch.empty(Kp * RS * Cp, dtype=dtype, device=w.device))
            pc.specs[key] = sp
        krsc, crsk = sp[7], sp[8]
    else:
        krsc = torch.empty(Kp * RS * Cp, dtype=dtype, device=w.device)
        crsk = torch.empty(Kp * RS * Cp, dtype=dtype, device=w.device)
    lib.adr_pack_weight2(dcode(dtype), fptr(wf), fptr(krsc), fptr(crsk), K, Kp, C, Cp, RS, transpose_kc, stream())
    return krsc, crsk


class WgradEntry(ctypes.Structure):
    """adr_wgrad_reduce_entry (include/adr.h)."""
    _fields_ = [("part", ctypes.c_void_p), ("dst", ctypes.c_void_p), ("split_stride", ctypes.c_long)] + [
        (n, ctypes.c_int) for n in ("splits", "K", "C", "Cp", "RS", "transpose_kc", "accumulate", "pad_")]


class WgradJob(ctypes.Structure):
    """adr_wgrad_job (include/adr.h)."""
    _fields_ = [("d", ConvDesc), ("x", ctypes.c_void_p), ("dy", ctypes.c_void_p), ("out", ctypes.c_void_p),
                ("accumulate", ctypes.c_int), ("pad_", ctypes.c_int), ("bias", ctypes.c_void_p)]


class PsumEntry(ctypes.Structure):
    """adr_psum_entry (include/adr.h)."""
    _fields_ = [("partial", ctypes.c_void_p), ("out", ctypes.c_void_p)] + [
        (n, ctypes.c_int) for n in ("P", "C", "which", "accumulate")]


class ColsumEntry(ctypes.Structure):
    """adr_colsum_entry (include/adr.h)."""
    _fields_ = [("x", ctypes.c_void_p), ("partial", ctypes.c_void_p)] + [
        (n, ctypes.c_int) for n in ("xcs", "N", "HW", "C", "rows_per_chunk", "chunks")]


class GnParamEntry(ctypes.Structure):
    """adr_gnparam_entry (include/adr.h)."""
    _fields_ = [(n, ctypes.c_void_p) for n in ("partial", "mean", "rstd", "dgamma", "dbeta")] + [
        (n, ctypes.c_int) for n in ("N", "chunks", "C", "G", "accumulate", "pad_")]


class DotsumEntry(ctypes.Structure):
    """adr_dotsum_entry (include/adr.h)."""
    _fields_ = [(n, ctypes.c_void_p) for n in ("x", "dz", "partial", "out")] + [
        (n, ctypes.c_int) for n in ("xcs", "dcs", "N", "HW", "C", "rows_per_chunk", "chunks", "pad_")]


class CopyPiece(ctypes.Structure):
    """adr_copy_piece (include/adr.h)."""
    _fields_ = [("src", ctypes.c_void_p), ("dst", ctypes.c_void_p)] + [
        (n, ctypes.c_int) for n in ("scs", "dcs", "C", "pad_")]


class AxpyEntry(ctypes.Structure):
    """adr_axpy_entry (include/adr.h)."""
    _fields_ = [("x", ctypes.c_void_p), ("y", ctypes.c_void_p), ("n", ctypes.c_long)]


def _nullctx():
    import contextlib
    return contextlib.nullcontext()


def _dbg_flush(kind, what):
    if _DEBUG_BNSTAT:
        import traceback
        print(f"deferral flush on repeated {kind} destination {what}:", "".join(traceback.format_stack(limit=5)[:-2]),
              flush=True)


class WgradDeferral:
    """Collects the split-K reductions of every conv weight gradient that lands in the trainer's gradient arena
    and runs them as a few batched launches (adr_wgrad_reduce_batched) when the backward pass ends, instead of
    one launch per conv. The partial slabs stay alive until then. A second entry for the same destination (a
    weight shared by several calls, e.g. the head's shared convs) flushes the pending batch first, so every
    destination's contributions still accumulate in program order."""

    def __init__(self):
        self.jobs, self.jkeep, self.jwork = [], [], []  # deferred WGRAD partial launches
        self.entries, self.keep, self.dsts = [], [], set()
        self.psums, self.pkeep, self.pdsts = [], [], set()
        self.axpys, self.akeep, self.adsts = [], [], set()
        self.cols, self.ckeep = [], []
        self.gnps, self.gkeep = [], []
        self.dots, self.dkeep = [], []
        self.post_dots = []  # callables run right after the batched dot sums (they consume their outputs)

    def add_dotsum(self, x, dy, out):
        """out[0] = sum(x * dy) over every pixel and channel (a scalar parameter gradient), at the flush.
        dy is pinned so no fan-out accumulates into it in place before then."""
        N, C, H, W = dy.shape
        vx, vd = _v(x), _v(dy)
        rows = _stats_rows(N, H * W)
        chunks = lib.adr_nc_reduce_chunks(H * W, rows)
        part = torch.empty(N * chunks * 2 * C, dtype=torch.float32, device=dy.device)
        vd[0]._adr_pinned = True
        dy._adr_pinned = True
        self.dots.append(DotsumEntry(vx[1], vd[1], part.data_ptr(), out.data_ptr(), vx[2], vd[2], N, H * W, C, rows,
                                     chunks, 0))
        self.dkeep += [vx[0], vd[0], part, out]

    def add_gnparam(self, part, mean, rstd, pg, pb, N, chunks, C, G, acc):
        """A GroupNorm dgamma / dbeta reduction (arena destinations), batched at the flush."""
        val = lambda q: q.value if isinstance(q, ctypes.c_void_p) else q  # noqa: E731
        self.gnps.append(GnParamEntry(part.data_ptr(), mean.data_ptr(), rstd.data_ptr(), val(pg), val(pb), N, chunks,
                                      C, G, acc, 0))
        self.gkeep += [part, mean, rstd]

    def add_colsum(self, x, part, xcs, N, HW, C, rows, chunks):
        """A bias gradient's column sums (adr_nc_reduce RED_STATS of dy into `part`), run in one batched launch
        before the partial sums at the flush; dy stays alive until then and is pinned (as in add_dotsum) so no
        fan-out sum accumulates into it in place before the flush reads it."""
        x._adr_pinned = True
        _v(x)[0]._adr_pinned = True
        self.cols.append(ColsumEntry(x.data_ptr(), part.data_ptr(), xcs, N, HW, C, rows, chunks))
        self.ckeep.append(x)
        self.ckeep.append(part)

    def add_axpy(self, src, dst, n):
        """A parameter gradient computed into a temporary, to be added into the arena (sink)."""
        dst = dst.value if isinstance(dst, ctypes.c_void_p) else int(dst)
        if dst in self.adsts:
            _dbg_flush("axpy", n)
            self.flush()
        self.axpys.append(AxpyEntry(src.data_ptr(), dst, n))
        self.akeep.append(src)
        self.adsts.add(dst)

    def add_psum(self, part, P, C, which, dst, acc):
        """A bias gradient (adr_partial_sum into the arena), batched the same way."""
        dst = dst.value if isinstance(dst, ctypes.c_void_p) else int(dst)
        if dst in self.pdsts:
            _dbg_flush("psum", C)
            self.flush()
        self.psums.append(PsumEntry(part.data_ptr(), dst, P, C, which, acc))
        self.pkeep.append(part)
        self.pdsts.add(dst)

    def add_job(self, d, xp, dyp, ws, keep, work=(0, 0), shp="", bias=None):
        """A conv's WGRAD partials into `ws`, launched at the flush together with the stage's other weight gradients
        (adr_conv2d_wgrad_partials_batched: one launch per tile shape, bitwise the per-conv launches). x and dy stay
        alive (keep) and dy is pinned so no fan-out accumulates into it in place before the flush reads it."""
        for t in keep:
            if torch.is_tensor(t):
                t._adr_pinned = True
                _v(t)[0]._adr_pinned = True
        self.jobs.append(WgradJob(ConvDesc.from_buffer_copy(d), xp, dyp, ws.data_ptr(), 0, 0,
                                  bias.data_ptr() if bias is not None else None))
        self.jwork.append((work, shp))
        self.jkeep += [ws, *keep] + ([bias] if bias is not None else [])

    def add(self, ws, stride, splits, dst, K_, C_, Cp, RS_, transpose_kc, acc):
        dst = dst.value if isinstance(dst, ctypes.c_void_p) else int(dst)
        if dst in self.dsts:
            _dbg_flush("wgrad", (K_, C_, RS_))
            self.flush()
        self.entries.append(WgradEntry(ws.data_ptr(), dst, stride, splits, K_, C_, Cp, RS_, transpose_kc, acc, 0))
        self.keep.append(ws)
        self.dsts.add(dst)

    def flush(self):
        self._flush()

    def _timed_jobs(self):
        """bench.py's roofline timing: the same grouped launches the step makes (one per tile shape, at most
        WGB_MAX = 24 jobs each), each bracketed by HIP events and labelled with the grouped kernel and the summed
        algorithmic bytes / flops of its jobs; thin / halo jobs (their own kernels) one call each. The partial
        writes are idempotent, so each call repeats TIMING_REPEAT times inside its event pair."""
        groups = {}
        for job, (work, shp) in zip(self.jobs, self.jwork):
            tile = lib.adr_conv2d_wgrad_batched_tile(ctypes.byref(job.d))
            groups.setdefault(tile, []).append((job, work, shp))
        for tile, items in groups.items():
            step = 24 if tile else 1
            for i in range(0, len(items), step):
                part = items[i:i + step]
                name = (f"void adr::wgrad_bf16_batched_kernel<{tile // 256}, {tile % 256}>(adr::WgBatch)" if tile
                        else "adr_conv2d_wgrad (thin / 3x3 halo kernel)")
                nb = sum(w[0] for _, w, _ in part)
                fl = sum(w[1] for _, w, _ in part)
                arr = (WgradJob * len(part))(*[j for j, _, _ in part])
                rep = TIMING_REPEAT
                tok = _t0(name, nb, fl, " + ".join(sh for _, _, sh in part), rep)
                for _ in range(rep):
                    lib.adr_conv2d_wgrad_partials_batched(ctypes.cast(arr, ctypes.c_void_p), len(part), stream())
                _t1(tok)

    def _flush(self):
        if self.jobs:  # the deferred weight-gradient partials, before their reductions
            if _TIMING is None:
                arr = (WgradJob * len(self.jobs))(*self.jobs)
                lib.adr_conv2d_wgrad_partials_batched(ctypes.cast(arr, ctypes.c_void_p), len(self.jobs), stream())
            else:
                self._timed_jobs()
            self.jobs, self.jkeep, self.jwork = [], [], []
        if self.dots:  # before the axpys that add their outputs into the arena
            arr = (DotsumEntry * len(self.dots))(*self.dots)
            lib.adr_dotsum_batched(ctypes.cast(arr, ctypes.c_void_p), len(self.dots), stream())
        for fn in self.post_dots:
            fn()
        if self.cols:  # before the partial sums that read their rows
            arr = (ColsumEntry * len(self.cols))(*self.cols)
            lib.adr_nc_reduce_batched(ctypes.cast(arr, ctypes.c_void_p), len(self.cols), stream())
        if self.entries:
            arr = (WgradEntry * len(self.entries))(*self.entries)
            lib.adr_wgrad_reduce_batched(ctypes.cast(arr, ctypes.c_void_p), len(self.entries), stream())
        if self.psums:
            arr = (PsumEntry * len(self.psums))(*self.psums)
            lib.adr_partial_sum_batched(ctypes.cast(arr, ctypes.c_void_p), len(self.psums), stream())
        if self.axpys:
            arr = (AxpyEntry * len(self.axpys))(*self.axpys)
            lib.adr_axpy_batched(ctypes.cast(arr, ctypes.c_void_p), len(self.axpys), stream())
        if self.gnps:
            arr = (GnParamEntry * len(self.gnps))(*self.gnps)
            lib.adr_gn_param_grad_batched(ctypes.cast(arr, ctypes.c_void_p), len(self.gnps), stream())
        self.entries, self.keep, self.dsts = [], [], set()
        self.psums, self.pkeep, self.pdsts = [], [], set()
        self.axpys, self.akeep, self.adsts = [], [], set()
        self.cols, self.ckeep = [], []
        self.gnps, self.gkeep = [], []
        self.dots, self.dkeep = [], []
        self.post_dots = []


def _defer_dot(param, x, dy):
    """Whether sum(x * dy) for a scalar parameter gradient can go to the deferral's batched flush."""
    return (_DEFER_DOT and _dfr() is not None and _TIMING is None and
            _target(param) is not None and dy.dtype == torch.bfloat16 and x.dtype == torch.bfloat16 and
            dy.shape[1] % 8 == 0 and _v(dy)[2] % 8 == 0 and _v(x)[2] % 8 == 0 and _v(dy)[1] % 16 == 0 and
            _v(x)[1] % 16 == 0)


# bias-gradient column sums batched at the flush (ADR_DEFER_COLSUM=0: one adr_nc_reduce per biased conv)
_DEFER_DOT = bool(int(__import__("os").environ.get("ADR_DEFER_DOT", "1")))  # scalar dot gradients at the flush
_DEFER_COLSUM = bool(int(__import__("os").environ.get("ADR_DEFER_COLSUM", "1")))
_DEFER = None  # the active WgradDeferral (set by the trainer around its backward pass)
# MLCA's two Conv1d weight gradients as partial sums at the flush (ADR_DEFER_MLCA=0: summed at the MLCA backward)
_DEFER_MLCA = bool(int(__import__("os").environ.get("ADR_DEFER_MLCA", "1")))
# Partial sets above this size are reduced right away (while still in L2) instead of deferred. Measured
# (scripts/ab_env.sh): deferring all of them is fastest — 32.39 ms vs 32.49 / 32.64 / 32.70 ms for 16 / 4 / 1 MB.
DEFER_MAX_BYTES = int(__import__("os").environ.get("ADR_DEFER_MAX_BYTES", 1 << 62))


def defer_wgrad():
    """Context manager: defer arena-bound WGRAD reductions to one batched flush at exit."""
    import contextlib

    @contextlib.contextmanager
    def _cm():
        global _DEFER
        prev, _DEFER = _DEFER, WgradDeferral()
        try:
            yield _DEFER
            _DEFER.flush()
        finally:
            _DEFER = prev
            bnxf_clear()
    return _cm()


def _dfr():
    """The active WgradDeferral (None outside a deferred backward)."""
    return _DEFER


def _grad_buf(tgt):
    """The gradient destination of arena parameter tgt: its arena slice."""
    return tgt._adr_grad


# WGRAD partials of arena-bound bf16 weight gradients deferred to the stage's flush and grouped into one launch per
# tile shape (WgradDeferral.add_job; ADR_DEFER_WGRAD=0: one launch per conv, at its backward)
_DEFER_WGRAD = bool(int(__import__("os").environ.get("ADR_DEFER_WGRAD", "1")))


def _fuse_wg_bias():
    """ADR_FUSE_WG_BIAS=0: bias gradients by their own column-sum pass (read per call: tests compare the two)."""
    return __import__("os").environ.get("ADR_FUSE_WG_BIAS", "1") != "0"


def _bias_rows(bias_param, K, P, part, device):
    """The fused bias gradient's [P][2][K] split rows into the parameter's gradient destination (batched at the
    flush when deferring; adr_partial_sum otherwise). Returns the autograd value (grad_ret)."""
    db, pb, acc = grad_dst(bias_param, K, device)
    if _dfr() is not None and acc:
        _dfr().add_psum(part, P, K, 0, pb, acc)
    else:
        lib.adr_partial_sum(fptr(part), P, K, 0, pb, acc, stream())
    return grad_ret(bias_param, db)


def wgrad_param(param, d, xp, dyp, K, C, RS, wshape, cpad, device, keep=(), bias=None):
    """Weight gradient of a conv contraction straight into its parameter's gradient destination: the split-K
    WGRAD GEMM writes [split][K][RS][C] fp32 slabs, and one fused reduce+unpack kernel sums the splits in a
    fixed order and scatters them into the (K, C, R, S) layout of `param` (the trainer's arena slice when
    present, accumulating; otherwise a fresh tensor returned for autograd). wshape may cover only the first
    rows / unpadded channels of the GEMM (padded convs, DCN's [Cout][9C] columns).
    bias: the conv's bias parameter — when given, returns (dw, fused, db): with fused True the bias gradient's column
    sums came out of the same deferred WGRAD launch (adr_wgrad_job.bias) and db is its autograd value."""
    K_, C_ = wshape[0], wshape[1]
    RS_ = 1
    for v in wshape[2:]:
        RS_ *= v
    return _wgrad_param(param, d, xp, dyp, K, C, RS, K_, C_, RS_, cpad, device, keep, bias)


def _wgrad_param(param, d, xp, dyp, K, C, RS, K_, C_, RS_, cpad, device, keep=(), bias=None):
    splits = lib.adr_conv2d_wgrad_splits(ctypes.byref(d))
    stride = K * RS * C
    es = 2 if d.dtype == BF16 else 4
    name = (f"void adr::wgrad_bf16_kernel<{_bn_of(K)}, {_bn_of(C)}>(adr::WgArgs)" if d.dtype == BF16
            else _gemm_symbol(F32, _bn_of(C), 2))
    work = (es * (d.n * d.h * d.w * d.c + d.n * d.ho * d.wo * d.k) + 4 * stride, 2 * d.n * d.ho * d.wo * d.k * RS * d.c)
    shp = _shape(d, f"wgrad/{splits}") if _TIMING is not None else ""
    ws = torch.empty(splits * stride, dtype=torch.float32, device=device)
    Cp = max(C_, cpad)
    out, ptr, acc = grad_dst(param, K_ * C_ * RS_, device)
    # the bias gradient's column sums from this same launch (deferred or not: the two paths stay bitwise equal)
    bpart = None
    if (bias is not None and d.dtype == BF16 and K == K_ and _fuse_wg_bias() and
            lib.adr_conv2d_wgrad_bias_fusable(ctypes.byref(d))):
        bpart = torch.empty(splits * 2 * K, dtype=torch.float32, device=device)

    def ret():
        if bias is None:
            return grad_ret(param, out)
        return (grad_ret(param, out), bpart is not None,
                _bias_rows(bias, K, splits, bpart, device) if bpart is not None else None)

    if (_DEFER_WGRAD and keep and _dfr() is not None and acc and d.dtype == BF16 and
            splits * stride * 4 <= DEFER_MAX_BYTES):
        # partials at the flush, grouped with the stage's other convs' (timed there per grouped launch)
        _dfr().add_job(d, xp, dyp, ws, keep, work, shp, bias=bpart)
        _dfr().add(ws, stride, splits, ptr, K_, C_, Cp, RS_, 0, acc)
        return ret()
    rep = _reps()
    tok = _t0(name, *work, shp, rep)
    for _ in range(rep):
        if bpart is not None:
            lib.adr_conv2d_wgrad_partials_bias(ctypes.byref(d), ctypes.c_void_p(xp), ctypes.c_void_p(dyp), fptr(ws),
                                               fptr(bpart), stream())
        else:
            lib.adr_conv2d_wgrad_partials(ctypes.byref(d), ctypes.c_void_p(xp), ctypes.c_void_p(dyp), fptr(ws), 0,
                                          stream())
    _t1(tok)
    if _dfr() is not None and acc and _TIMING is None and splits * stride * 4 <= DEFER_MAX_BYTES:
        _dfr().add(ws, stride, splits, ptr, K_, C_, Cp, RS_, 0, acc)
        return ret()
    tok = _t0("adr::wgrad_reduce_kernel<true, OUT, SL> (split reduce + unpack)",
              4 * stride * (splits + 1), stride * splits, shp)
    lib.adr_wgrad_reduce_unpack(fptr(ws), stride, splits, ptr, K_, C_, Cp, RS_, 0, acc, stream())
    _t1(tok)
    return ret()


def _bias_grad(dy, K, N, HW, cs, param=None):
    """Per-channel sum of dy. With `param`, accumulates into its gradient destination (grad_dst) and returns
    the autograd value; otherwise returns a fresh (K,) tensor."""
    return _bias_grad1(dy, K, N, HW, cs, param)


def _bias_grad1(dy, K, N, HW, cs, param=None):
    dt = dcode(dy.dtype)
    chunks = lib.adr_nc_reduce_chunks(HW, _stats_rows(N, HW))
    part = torch.empty(N * chunks * 2 * K, dtype=torch.float32, device=dy.device)
    if param is not None and _dfr() is not None and _TIMING is None and _DEFER_COLSUM and dt == BF16 and \
            dy.data_ptr() % 16 == 0 and cs % 8 == 0 and K % 8 == 0 and \
            _target(param) is not None:  # an arena destination: column sums and partial sums at the flush, batched
        db, p, acc = grad_dst(param, K, dy.device)
        _dfr().add_colsum(dy, part, cs, N, HW, K, _stats_rows(N, HW), chunks)
        _dfr().add_psum(part, N * chunks, K, 0, p, acc)
        return grad_ret(param, db)
    lib.adr_nc_reduce(dt, 0, ctypes.c_void_p(dy.data_ptr()), cs, 0, None, 0, 0, None, None, 0, 0, N, HW, K,
                      _stats_rows(N, HW), fptr(part), stream())
    if param is not None:
        db, p, acc = grad_dst(param, K, dy.device)
        if _dfr() is not None and acc and _TIMING is None:
            _dfr().add_psum(part, N * chunks, K, 0, p, acc)
        else:
            lib.adr_partial_sum(fptr(part), N * chunks, K, 0, p, acc, stream())
        return grad_ret(param, db)
    db = torch.empty(K, dtype=torch.float32, device=dy.device)
    lib.adr_partial_sum(fptr(part), N * chunks, K, 0, fptr(db), 0, stream())
    return db


def _conv_fwd_bnact(ctx, pend, w, stride, pad, want_stats, box):
    """Conv2dFn's forward on a pending BN-act input (BnFwd): one adr_conv2d_fwd_bf16_bnact launch reads y, applies
    z = act(y * s + t) while staging, side-writes z and computes the conv (+ BN partial statistics). Returns
    (None, None) when the fused kernel would stage each element more than BN_XF_MAX_REUSE / 100 times (then the
    caller writes z first and runs the plain conv)."""
    z = pend.z
    y, yp, ycs = nhwc(pend.y)
    N, C, H, W = y.shape
    K, Cw, R, S = w.shape
    if Cw != C:
        raise RuntimeError(f"Conv2dFn: input has {C} channels, weight expects {Cw}")
    (sh, sw), (ph, pw) = _pair(stride), _pair(pad)
    Ho, Wo = (H + 2 * ph - R) // sh + 1, (W + 2 * pw - S) // sw + 1
    d, Ho, Wo = conv_desc(N, H, W, C, ycs, K, R, S, sh, sw, ph, pw, K, torch.bfloat16)
    if not _engine2(d, d.c) or lib.adr_conv2d_bf16_xf_reuse(ctypes.byref(d), 0) > BN_XF_FWD_MAX_REUSE:
        pend.materialize()
        return None, None
    wp, wt = pack_weight2(w, torch.bfloat16)
    out, op, ocs = _out_view(box, N, K, Ho, Wo, torch.bfloat16, y.device)
    d.y_cstride = ocs
    stats = None
    if want_stats:
        stats = torch.empty(lib.adr_conv2d_fwd_bf16_bnact_stat_tiles(ctypes.byref(d)) * 2 * K, dtype=torch.float32,
                            device=y.device)
    st = pend.struct()
    pend.done()
    sym = "" if _TIMING is None else _conv2_symbol(d, 2)
    tok = _t0(sym, *_conv_work(d), _shape(d, "fwd+bnact") if _TIMING is not None else "")
    lib.adr_conv2d_fwd_bf16_bnact(ctypes.byref(d), ctypes.c_void_p(yp), ctypes.c_void_p(wp.data_ptr()),
                                  ctypes.c_void_p(op), fptr(stats), ctypes.byref(st), stream())
    _t1(tok)
    ctx.act = None
    ctx.save_for_backward(z, wp, wt, None)
    ctx.meta = (stride, pad, 0, w.shape, False)
    ctx.pw, ctx.pb = w, None
    if stats is None:
        stats = torch.empty(0, device=y.device)
    ctx.mark_non_differentiable(stats)
    return (out if box is None else out[:, :]), stats


class Conv2dFn(torch.autograd.Function):
    """y = conv2d(x, w) + b (dense, groups=1). Optionally also returns per-tile BN partial statistics."""

    @staticmethod
    def forward(ctx, x, w, b, stride, pad, want_stats, cpad, box=None, act=None):
        ctx.set_materialize_grads(False)  # no zero-filled gradient for the statistics output
        sink = getattr(x, "_adr_sink", None)
        ctx.sink = sink if sink is not None and sink.fits(x) else None
        dtype = x.dtype
        pend = _bnf_of(x)  # x = act(bn(y)) not written yet: stage y through the BN-act here
        # this conv is the only reader of a lazy BN-act output: its data gradient is that BN's complete dz, so the
        # BN's backward statistics can come from the dgrad epilogue (BnStat / BSTAT)
        ctx.bstat = pend.bstat if pend is not None and pend.bstat is not None and not pend.bstat.shared else None
        if pend is not None and not (b is None and act is None and cpad == 0 and not CONV_FP8):
            pend.materialize()
            pend = None
        if pend is not None:
            y, stats = _conv_fwd_bnact(ctx, pend, w, stride, pad, want_stats, box)
            if y is not None:
                return y, stats
            pend = None
        x, xp, xcs = nhwc(x)
        N, C, H, W = x.shape
        K, Cw, R, S = w.shape
        Cp = max(Cw, cpad)
        if C != Cp:
            raise RuntimeError(f"Conv2dFn: input has {C} channels, weight expects {Cw} (padded {Cp})")
        wp, wt = pack_weight2(w, dtype, cpad)
        (sh, sw), (ph, pw) = _pair(stride), _pair(pad)
        Ho, Wo = (H + 2 * ph - R) // sh + 1, (W + 2 * pw - S) // sw + 1
        y, yp, ycs = _out_view(box, N, K, Ho, Wo, dtype, x.device)  # a concat slice when the caller boxes one
        d, Ho, Wo = conv_desc(N, H, W, C, xcs, K, R, S, sh, sw, ph, pw, ycs, dtype)
        stats = None
        if want_stats:
            tiles = (lib.adr_conv2d_fwd_bf16_stat_tiles if _engine2(d, d.c) else
                     lib.adr_conv2d_fwd_stat_tiles)(ctypes.byref(d))
            stats = torch.empty(tiles * 2 * K, dtype=torch.float32, device=x.device)
        bf = b.detach().float().contiguous() if b is not None else None
        # fp8 for the Conv-BN-act convs only: biased nn.Conv2d rows (the heads' output projections: logits, box
        # bins, offsets) stay bf16, as fp8 training recipes keep the output layers in higher precision
        if CONV_FP8 and b is None and act is None and dtype == torch.bfloat16 and C >= _FP8_MIN_C and R * S > 1 and \
                lib.adr_conv2d_fp8_supported(ctypes.byref(d)):
            if want_stats:  # the fp8 engine tiles every geometry by 128 output rows
                stats = torch.empty(lib.adr_conv2d_fwd_fp8_stat_tiles(ctypes.byref(d)) * 2 * K, dtype=torch.float32,
                                    device=x.device)
            conv_fwd_fp8(d, xp, w, Cw, Cp, bf, yp, stats)
        elif act is not None:  # act(conv + b) on the fp32 accumulator (conv_act checked the engine)
            conv_fwd_act(d, xp, wp.data_ptr(), bf, K, act, yp)
        else:
            conv_fwd(d, xp, wp.data_ptr(), fptr(bf), yp, fptr(stats))
        ctx.act = act
        ctx.save_for_backward(x, wp, wt, y if act is not None else None)  # the activation's backward reads its output
        ctx.meta = (stride, pad, cpad, w.shape, b is not None)
        ctx.pw, ctx.pb = w, b
        if stats is None:
            stats = torch.empty(0, device=x.device)
        ctx.mark_non_differentiable(stats)
        return (y if box is None else y[:, :]), stats

    @staticmethod
    def backward(ctx, dy, _dstats):
        if dy is None:
            return None, None, None, None, None, None, None, None, None
        x, wp, wt, z = ctx.saved_tensors
        stride, pad, cpad, wshape, has_b = ctx.meta
        (sh, sw), (ph, pw) = _pair(stride), _pair(pad)
        if ctx.act is not None:  # dy of the pre-activation from the saved output (torch sigmoid/threshold_backward)
            dz = dy.to(x.dtype) if dy.dtype != x.dtype else dy
            dy = _new_like(z)
            _ew(EW_ACT_BWD_OUT, _v(dy), _v(z), _v(dz), act=ACT[ctx.act])
        pend = BnXf.take(dy)  # an unwritten BN-act backward (BNActFn with xfuse): dz + coefficients
        dy, dyp, dycs = nhwc(dy.to(x.dtype) if dy.dtype != x.dtype else dy)
        N, C, H, W = x.shape
        K, _, R, S = wshape
        x, xp, xcs = nhwc(x)
        d, Ho, Wo = conv_desc(N, H, W, C, xcs, K, R, S, sh, sw, ph, pw, dycs, x.dtype)
        dx = dw = db = None
        if pend is not None:
            d2, _, _ = conv_desc(N, H, W, C, C, K, R, S, sh, sw, ph, pw, dycs, x.dtype)
            if not (ctx.needs_input_grad[0] and wt is not None and _engine2(d2, d2.k) and d2.stride_h in (1, 2) and
                    lib.adr_conv2d_bf16_xf_reuse(ctypes.byref(d2), 1) <= BN_XF_MAX_REUSE):
                pend.materialize(dy)  # no fused data gradient for this conv: write dy first
                pend = None
        if ctx.needs_input_grad[0]:
            d2, _, _ = conv_desc(N, H, W, C, C, K, R, S, sh, sw, ph, pw, dycs, x.dtype)
            if ctx.sink is not None:  # into the fan-out's shared gradient (accumulating after the first consumer)
                buf, acc, add = ctx.sink.claim(x.device, can_add=wt is not None and _engine2(d2, d2.k))
                if buf.stride(3) != C:  # a seeded concat-gradient slice: the concat's channel stride
                    d2, _, _ = conv_desc(N, H, W, C, buf.stride(3), K, R, S, sh, sw, ph, pw, dycs, x.dtype)
                conv_dgrad(d2, dyp, (wp, wt), None, buf.data_ptr(), accumulate=acc, addend=add, xf=pend, dy=dy)
            else:
                dx = empty_act(N, C, H, W, x.dtype, x.device)
                bst = ctx.bstat if (ctx.bstat is not None and BN_BSTAT and wt is not None and _engine2(d2, d2.k)
                                    and d2.stride_h in (1, 2) and x.dtype == torch.bfloat16) else None
                conv_dgrad(d2, dyp, (wp, wt), None, dx.data_ptr(), xf=pend, dy=dy, bst=bst, dx=dx)
        fused = False
        if ctx.needs_input_grad[1]:
            if has_b and ctx.needs_input_grad[2]:  # the bias column sums from the same WGRAD launch when it can
                dw, fused, db = wgrad_param(ctx.pw, d, xp, dyp, K, C, R * S, wshape, cpad, x.device, keep=(x, dy),
                                            bias=ctx.pb)
            else:
                dw = wgrad_param(ctx.pw, d, xp, dyp, K, C, R * S, wshape, cpad, x.device, keep=(x, dy))
        if has_b and ctx.needs_input_grad[2] and not fused:
            db = _bias_grad(dy, K, N, Ho * Wo, dycs, ctx.pb)
        return dx, dw, db, None, None, None, None, None, None


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
        wp, wt = pack_weight2(w, dtype)  # (Ci, Co, R, S) == KRSC of the equivalent conv (K=Ci, C=Co)
        y = empty_act(N, Co, Ho, Wo, dtype, x.device)
        d, h2, w2 = conv_desc(N, Ho, Wo, Co, Co, Ci, R, S, stride, stride, pad, pad, xcs, dtype)
        if (h2, w2) != (H, W):
            raise RuntimeError("ConvT2dFn: inconsistent geometry")
        bf = b.detach().float().contiguous() if b is not None else None
        conv_dgrad(d, xp, (wp, wt), fptr(bf), y.data_ptr())
        ctx.save_for_backward(x, wp)
        ctx.meta = (stride, pad, w.shape, b is not None, Ho, Wo)
        ctx.pw, ctx.pb = w, b
        return y

    @staticmethod
    def backward(ctx, dy):
        x, wp = ctx.saved_tensors
        stride, pad, wshape, has_b, Ho, Wo = ctx.meta
        dy, dyp, dycs = nhwc(dy.to(x.dtype) if dy.dtype != x.dtype else dy)
        x, xp, xcs = nhwc(x)
        N, Ci, H, W = x.shape
        _, Co, R, S = wshape
        dx = dw = db = None
        if ctx.needs_input_grad[0]:
            dx = empty_act(N, Ci, H, W, x.dtype, x.device)
            d, _, _ = conv_desc(N, Ho, Wo, Co, dycs, Ci, R, S, stride, stride, pad, pad, Ci, x.dtype)
            conv_fwd(d, dyp, wp.data_ptr(), None, dx.data_ptr())
        if ctx.needs_input_grad[1]:
            # equivalent conv: input = dy_T (N, Ho, Wo, Co), output grad = x_T (N, H, W, Ci)
            d, _, _ = conv_desc(N, Ho, Wo, Co, dycs, Ci, R, S, stride, stride, pad, pad, xcs, x.dtype)
            dw = wgrad_param(ctx.pw, d, dyp, xp, Ci, Co, R * S, wshape, 0, x.device, keep=(x, dy))
        if has_b and ctx.needs_input_grad[2]:
            db = _bias_grad(dy, Co, N, Ho * Wo, dycs, ctx.pb)
        return dx, dw, db, None, None, None


class BNActFn(torch.autograd.Function):
    """act(BatchNorm2d(y)) — train mode uses batch statistics (from the conv epilogue when given)."""

    @staticmethod
    def forward(ctx, y, stats, gamma, beta, rm, rv, act, training, momentum, eps, box=None, xfuse=False, lazy=False,
                res=None):
        dtype = y.dtype
        y, yp, ycs = nhwc(y)
        N, C, H, W = y.shape
        HW = H * W
        dev = y.device
        # the backward may hand its dy to the producing conv unmaterialised (see BnXf): y must come from a dense conv
        # whose only reader is this BN (Conv.forward), on the bf16 engine's XF coefficient table
        ctx.xfuse = bool(xfuse) and BN_XF_BWD and training and dtype == torch.bfloat16 and act in ("silu", "none") \
            and C <= 512 and C % 8 == 0
        f = lambda: torch.empty(C, dtype=torch.float32, device=dev)  # noqa: E731
        scale, shift, mean, rstd = f(), f(), f(), f()
        if training:
            if stats is None or stats.numel() == 0:
                chunks = lib.adr_nc_reduce_chunks(HW, _stats_rows(N, HW))
                stats = torch.empty(N * chunks * 2 * C, dtype=torch.float32, device=dev)
                lib.adr_nc_reduce(dcode(dtype), 0, ctypes.c_void_p(yp), ycs, 0, None, 0, 0, None, None, 0, 0,
                                  N, HW, C, _stats_rows(N, HW), fptr(stats), stream())
            P = stats.numel() // (2 * C)
        else:
            P = 0
        lib.adr_bn_finalize(fptr(stats) if training else None, P, C, float(N * HW), fptr(gamma.detach()),
                            fptr(beta.detach()), fptr(rm), fptr(rv), float(momentum),
                            float(eps), int(training), fptr(scale), fptr(shift), fptr(mean), fptr(rstd), stream())
        z, zp, zcs = _out_view(box, N, C, H, W, dtype, dev)
        ctx.sres = getattr(res, "_adr_sink", None) if res is not None else None
        ctx.bstat = None
        if res is not None:  # z = act(bn(y)) + res: the residual add in the same pass
            vr = _v(res)
            lib.adr_affine_act_res(dcode(dtype), ctypes.c_void_p(yp), ycs, 0, ctypes.c_void_p(vr[1]), vr[2],
                                   ctypes.c_void_p(zp), zcs, 0, fptr(scale), fptr(shift), 0, ACT[act], N, HW, C,
                                   stream())
        elif lazy and box is None and BN_XF_FWD and training and dtype == torch.bfloat16 and act in ("silu", "none") \
                and C % 8 == 0 and C <= 512:
            # z is written by its consumer conv (or on first other read); that conv, z's only reader, also takes the
            # BN's backward statistics in its data gradient's epilogue (BnStat)
            ctx.bstat = BnStat(y, scale, shift, act) if BN_BSTAT else None
            BnFwd(y, scale, shift, act, z, ctx.bstat).attach()
        else:
            lib.adr_affine_act(dcode(dtype), ctypes.c_void_p(yp), ycs, 0, ctypes.c_void_p(zp), zcs, 0,
                               fptr(scale), fptr(shift), 0, ACT[act], N, HW, C, stream())
        ctx.save_for_backward(y, scale, shift, mean, rstd, gamma)
        ctx.meta = (act, training)
        ctx.pbeta = beta
        return z

    @staticmethod
    def backward(ctx, dz):
        y, scale, shift, mean, rstd, gamma = ctx.saved_tensors
        act, training = ctx.meta
        # the statistics partials the consumer conv's data gradient wrote with dz (BSTAT), when dz is that buffer
        got = ctx.bstat.take(dz) if ctx.bstat is not None else None
        ctx.bstat = None
        dz, dzp, dzcs = nhwc(dz.to(y.dtype) if dz.dtype != y.dtype else dz)
        # the residual's gradient is dz itself (held for a conv consumer's dgrad epilogue when its fan-out allows)
        dres = _defer_pass(ctx.sres, dz) if ctx.needs_input_grad[13] else None
        _, yp, ycs = nhwc(y)
        N, C, H, W = y.shape
        HW = H * W
        dev = y.device
        dt = dcode(y.dtype)
        chunks = lib.adr_nc_reduce_chunks(HW, _stats_rows(N, HW))
        part = torch.empty(N * chunks * 2 * C, dtype=torch.float32, device=dev) if got is None else None
        f = lambda: torch.empty(C, dtype=torch.float32, device=dev)  # noqa: E731
        A, B, Cc = f(), f(), f()
        dgamma, pg, acc_g = grad_dst(gamma, C, dev)
        dbeta, pb, acc_b = grad_dst(ctx.pbeta, C, dev)
        if acc_g != acc_b:
            raise RuntimeError("BN gamma/beta gradients must share one destination kind")
        if got is not None:
            part, P = got
        else:
            P = N * chunks
            if _DEBUG_BNSTAT:
                print(f"BN bwd stats pass: dz from {getattr(dz, '_adr_src', '?')} {tuple(dz.shape)} act {act} "
                      f"xfuse {ctx.xfuse} sres {ctx.sres is not None}", flush=True)
            lib.adr_nc_reduce(dt, 1, ctypes.c_void_p(yp), ycs, 0, ctypes.c_void_p(dzp), dzcs, 0, fptr(scale),
                              fptr(shift), 0, ACT[act], N, HW, C, _stats_rows(N, HW), fptr(part), stream())
        lib.adr_bn_bwd_finalize(fptr(part), P, C, float(N * HW), fptr(mean), fptr(rstd),
                                fptr(gamma.detach()), pg, pb, fptr(A), fptr(B), fptr(Cc), int(training), acc_g,
                                stream())
        dy = empty_act(N, C, H, W, y.dtype, dev)
        pend = BnXf(y, dz, scale, shift, A, B, Cc, act)
        if ctx.xfuse:  # the conv's data gradient applies it while staging its operand (and side-writes dy)
            pend.attach(dy)
        else:
            pend.materialize(dy)
        return (dy, None, grad_ret(gamma, dgamma), grad_ret(ctx.pbeta, dbeta), None, None, None, None, None, None, None,
                None, None, dres)


# Training Conv-BN-act backward fusion: BNActFn.backward computes the coefficients (nc_reduce + bn_bwd_finalize)
# but leaves dy = A * dz * act'(y * s + t) + B * y + C unwritten; the producing conv's Conv2dFn.backward runs its
# data gradient on dz with that transform in the operand staging (adr_conv2d_dgrad_bf16_bnact), which also writes
# dy once for the weight gradient — the affine_act_bwd pass and its launch disappear. ADR_BN_XF_BWD=0 disables.
BN_XF_BWD = bool(int(__import__("os").environ.get("ADR_BN_XF_BWD", "1")))
# The transform is VALU work per staged operand element (a sigmoid for SiLU): measured, the fused data gradient of a
# 3x3 implicit-GEMM conv (each dz element staged 9x) or of a multi-column-tile 1x1 ran 3x slower than the
# affine_act_bwd + dgrad pair, so the fusion is taken only where each element is staged about once (x100)
BN_XF_MAX_REUSE = int(__import__("os").environ.get("ADR_BN_XF_MAX_REUSE", "150"))
# data_ptr -> (BnXf, dy): unwritten dy buffers handed to a conv backward. The entry holds dy itself, so its memory
# cannot be reused by another tensor while the entry exists; entries nobody consumed (a frozen producing conv) are
# dropped at the end of the backward (defer_wgrad's exit, bnxf_clear)
_BNXF_PENDING = {}


# Training Conv-BN-act forward fusion: BNActFn (lazy) computes the batch statistics and coefficients but leaves
# z = act(y * s + t) unwritten; the consumer conv (Conv2dFn) stages y through the transform
# (adr_conv2d_fwd_bf16_bnact: streaming 1x1 / 3x3 halo tiles / implicit GEMM) and side-writes z once for the
# layer's weight gradient — the affine_act pass (a read of y, a launch) disappears. Taken where the consumer stages
# each element about once (BN_XF_MAX_REUSE); any other reader of a pending z writes it first (nhwc -> _bnf_settle).
# ADR_BN_XF_FWD=0 disables.
BN_XF_FWD = bool(int(__import__("os").environ.get("ADR_BN_XF_FWD", "1")))
# the forward transform is one affine + activation per staged element (the backward's needs a second operand and
# the BN-backward linear term): two column tiles of the streaming 1x1 kernel still qualify
BN_XF_FWD_MAX_REUSE = int(__import__("os").environ.get("ADR_BN_XF_FWD_MAX_REUSE", "200"))
_BNF_PENDING = {}  # storage data_ptr -> BnFwd


class BnFwd:
    """A pending BN-act forward: z (allocated, unwritten) = act(y * scale + shift); bstat: the BN's BnStat."""
    __slots__ = ("y", "scale", "shift", "act", "z", "key", "bstat")

    def __init__(self, y, scale, shift, act, z, bstat=None):
        self.y, self.scale, self.shift, self.act, self.z = y, scale, shift, act, z
        self.bstat = bstat
        self.key = z.untyped_storage().data_ptr()

    def attach(self):
        _BNF_PENDING[self.key] = self

    def done(self):
        _BNF_PENDING.pop(self.key, None)

    def materialize(self):
        self.done()
        y, yp, ycs = nhwc(self.y)
        z, zp, zcs = nhwc(self.z)
        N, C, H, W = y.shape
        lib.adr_affine_act(dcode(y.dtype), ctypes.c_void_p(yp), ycs, 0, ctypes.c_void_p(zp), zcs, 0, fptr(self.scale),
                           fptr(self.shift), 0, ACT[self.act], N, H * W, C, stream())

    def struct(self):
        _, yp, ycs = nhwc(self.y)
        return BnXfStruct(yp, self.scale.data_ptr(), self.shift.data_ptr(), None, None, None, self.z.data_ptr(), ycs,
                          self.z.stride(1) if self.z.shape[1] == 1 else self.z.stride(3), ACT[self.act], 0)


def _bnf_settle(t):
    """Write a pending BN-act output before t (it, or a view of its storage) is read."""
    try:
        key = t.untyped_storage().data_ptr()
    except RuntimeError:
        return
    p = _BNF_PENDING.get(key)
    if p is not None:
        if p.bstat is not None:  # z has another reader: the consumer conv's dgrad is not its whole gradient
            p.bstat.shared = True
        p.materialize()


def _bnf_of(x):
    """The pending BN-act forward whose output is exactly x (whole tensor, same view), or None. A partial view of a
    pending output is written first (nhwc) instead."""
    if not _BNF_PENDING or not x.is_cuda:
        return None
    p = _BNF_PENDING.get(x.untyped_storage().data_ptr())
    if p is None:
        return None
    z = p.z
    if x.data_ptr() == z.data_ptr() and x.shape == z.shape and x.stride() == z.stride():
        return p
    return None


def bnf_clear():
    """Write every pending BN-act output (end of a forward: nothing may stay unwritten)."""
    for p in list(_BNF_PENDING.values()):
        p.materialize()


def bnf_drop():
    """Forget every pending BN-act output without writing it (a forward that raised part-way: launching their
    affine_act later could land inside the next forward or graph capture; the entries also pin y and z)."""
    _BNF_PENDING.clear()


def bnxf_clear():
    """Drop pending BN-act backward entries no conv consumed (end of a backward pass)."""
    _BNXF_PENDING.clear()


# BN backward statistics in the consumer's data gradient (BSTAT): a lazy BN-act output z (kernels.BnFwd) has exactly
# one reader, the conv that stages it, so that conv's data gradient IS the BN's complete dz. Its epilogue reads y
# alongside and writes the (sum g, sum g * y) partials adr_nc_reduce's backward pass would (adr_conv2d_dgrad_bf16_bstat),
# and BNActFn.backward finalizes from them: the nc_reduce launch and its read of dz and y disappear. The sums are
# the same per-element terms in another order (fixed per geometry: deterministic). ADR_BN_BSTAT=0 disables.
BN_BSTAT = bool(int(__import__("os").environ.get("ADR_BN_BSTAT", "1")))


class BStatStruct(ctypes.Structure):
    """adr_bn_bstat (include/adr.h)."""
    _fields_ = [("y", ctypes.c_void_p), ("scale", ctypes.c_void_p), ("shift", ctypes.c_void_p),
                ("y_cstride", ctypes.c_int), ("act", ctypes.c_int)]


_DEBUG_BNSTAT = bool(int(__import__("os").environ.get("ADR_DEBUG_BNSTAT", "0")))


class BnStat:
    """A training BN-act's backward statistics, taken from its only reader's data gradient: (y, scale, shift, act)
    from the forward; after that dgrad, the partials and the identity (address, geometry, version) of the dz
    buffer they were computed from — BNActFn.backward uses them only for exactly that, unmodified, buffer."""
    __slots__ = ("y", "scale", "shift", "act", "shared", "part", "P", "key", "ref")

    def __init__(self, y, scale, shift, act):
        self.y, self.scale, self.shift, self.act = y, scale, shift, act
        self.shared = False
        self.part = self.P = self.key = self.ref = None

    def struct(self):
        _, yp, ycs = nhwc(self.y)
        return BStatStruct(yp, self.scale.data_ptr(), self.shift.data_ptr(), ycs, ACT[self.act])

    @staticmethod
    def _key(t):
        return t.data_ptr(), tuple(t.shape), tuple(t.stride()), t.dtype, t._version

    def set(self, part, P, dx):
        # a weak reference to dx itself: a buffer freed and re-allocated at the same address is not dx
        self.part, self.P, self.key, self.ref = part, P, self._key(dx), weakref.ref(dx)

    def take(self, dz):
        """(partials, rows) when dz is the buffer the dgrad wrote them with (else None): dx still alive, dz the
        same storage at the same geometry and version; clears the holder."""
        dx = self.ref() if self.ref is not None else None
        ok = (dx is not None and self._key(dz) == self.key and
              (dz is dx or dz.untyped_storage().data_ptr() == dx.untyped_storage().data_ptr()))
        if _DEBUG_BNSTAT and self.key is not None and not ok:
            print(f"BnStat.take miss: key {'same' if self._key(dz) == self.key else 'differs'}, dx "
                  f"{'dead' if dx is None else 'alive'} {tuple(dz.shape)}", flush=True)
        got = (self.part, self.P) if ok else None
        self.part = self.P = self.key = self.ref = None
        return got


class BnXfStruct(ctypes.Structure):
    """adr_bnact_xf (include/adr.h)."""
    _fields_ = [(n, ctypes.c_void_p) for n in ("y", "scale", "shift", "A", "B", "Cc", "out")] + [
        (n, ctypes.c_int) for n in ("y_cstride", "out_cstride", "act", "pad_")]


class BnXf:
    """A pending BN-act backward: dy (the buffer it is attached to) = A * g + B * y + C, g = dz * act'(y*s + t)."""
    __slots__ = ("y", "dz", "scale", "shift", "A", "B", "Cc", "act")

    def __init__(self, y, dz, scale, shift, A, B, Cc, act):
        self.y, self.dz, self.scale, self.shift, self.A, self.B, self.Cc, self.act = y, dz, scale, shift, A, B, Cc, act

    def attach(self, dy):
        _BNXF_PENDING[dy.data_ptr()] = (self, dy)
        dy._adr_bnxf = self

    @staticmethod
    def take(dy):
        """The pending transform of a gradient buffer handed to a conv backward (removed from the registry). A
        tensor object that lost the attribute (autograd re-wrapped it) matches its entry only when it is a view of
        exactly the registered buffer: same address, shape, strides and dtype."""
        p = getattr(dy, "_adr_bnxf", None)
        ent = _BNXF_PENDING.get(dy.data_ptr())
        if p is None and ent is not None:
            t = ent[1]
            if t.shape == dy.shape and t.stride() == dy.stride() and t.dtype == dy.dtype:
                p = ent[0]
        if p is not None:
            if ent is not None and ent[0] is p:
                del _BNXF_PENDING[dy.data_ptr()]
            try:
                del dy._adr_bnxf
            except AttributeError:
                pass
        return p

    def materialize(self, dy):
        """Write dy with adr_affine_act_bwd (the unfused path)."""
        y, yp, ycs = nhwc(self.y)
        _, dzp, dzcs = nhwc(self.dz)
        N, C, H, W = y.shape
        lib.adr_affine_act_bwd(dcode(y.dtype), ctypes.c_void_p(yp), ycs, 0, ctypes.c_void_p(dzp), dzcs, 0,
                               ctypes.c_void_p(dy.data_ptr()), dy.stride(3), 0, fptr(self.scale), fptr(self.shift),
                               fptr(self.A), fptr(self.B), fptr(self.Cc), 0, 0, ACT[self.act], N, H * W, C, 0,
                               stream())

    def struct(self, dy):
        _, yp, ycs = nhwc(self.y)
        return BnXfStruct(yp, self.scale.data_ptr(), self.shift.data_ptr(), self.A.data_ptr(), self.B.data_ptr(),
                          self.Cc.data_ptr(), dy.data_ptr(), ycs, dy.stride(3), ACT[self.act], 0)


_GN_FUSED = bool(int(__import__("os").environ.get("ADR_GN_FUSED", "1")))  # 0: the 3-launch path (A/B, parity)
# one workgroup per image streams the image twice from one CU: past ~40x40 maps the three-launch path (the whole
# chip on every pass) is faster
_GN_FUSED_MAXHW = int(__import__("os").environ.get("ADR_GN_FUSED_MAXHW", "400"))


_DEFER_GN = bool(int(__import__("os").environ.get("ADR_DEFER_GN", "1")))  # 0: GN param grads launched in place


def _defer_gn(acc):
    """Whether a GroupNorm dgamma / dbeta reduction goes to the deferral's batched flush (arena destinations)."""
    return bool(acc) and _DEFER_GN and _dfr() is not None and _TIMING is None


_GATE_GRAD = {}  # dy.data_ptr() -> (weakref to dy, dgate): per-image gate gradients computed by a GN backward
_GN_GATE = bool(int(__import__("os").environ.get("ADR_GN_GATE", "1")))  # 0: gate gradient from sum(dy * out) (A/B)


def _gn_gate_grad(gate, eps, part, ks, N, chunks, sub_rows, C, groups, gammas, mean, rstd, dy):
    """dL/ds of the per-image gate s whose output s*y this GroupNorm normalised (ScaleFn grad_from_out), from the
    GN backward's own fp32 partial rows (adr_gn_gate_grad: the exact eps residue of the scale-invariant sum), left
    for ScaleFn.backward under dy's address."""
    dgate = torch.empty_like(gate)
    kk = (ctypes.c_int * len(ks))(*ks)
    gp, _keep = _ptrs(gammas)
    lib.adr_gn_gate_grad(fptr(part), len(ks), ctypes.cast(kk, ctypes.c_void_p), N, chunks, sub_rows, C, groups, gp,
                         fptr(mean), fptr(rstd), float(eps), fptr(gate), fptr(dgate), stream())
    for key in [key for key, (r, _) in _GATE_GRAD.items() if r() is None]:
        del _GATE_GRAD[key]
    _GATE_GRAD[dy.data_ptr()] = (weakref.ref(dy), dgate)


class GNActFn(torch.autograd.Function):
    """act(GroupNorm(G)(y)) with per-(image, group) statistics."""

    @staticmethod
    def forward(ctx, y, gamma, beta, groups, act, eps):
        dtype = y.dtype
        ctx.gate, ctx.eps = getattr(y, "_adr_gate", None) if _GN_GATE else None, eps  # y = s*conv() (ScaleFn)
        y, yp, ycs = nhwc(y)
        N, C, H, W = y.shape
        HW = H * W
        dev = y.device
        ctx.fused = _GN_FUSED and HW <= _GN_FUSED_MAXHW and bool(lib.adr_gn_fused_supported(dcode(dtype), C, groups))
        if ctx.fused:  # one launch per layer: a workgroup per image does statistics + affine + activation
            scale = torch.empty(N * C, dtype=torch.float32, device=dev)
            shift = torch.empty(N * C, dtype=torch.float32, device=dev)
            mean = torch.empty(N * groups, dtype=torch.float32, device=dev)
            rstd = torch.empty(N * groups, dtype=torch.float32, device=dev)
            z = empty_act(N, C, H, W, dtype, dev)
            lib.adr_gn_act_fused(dcode(dtype), ctypes.c_void_p(yp), ycs, 0, ctypes.c_void_p(z.data_ptr()), C, 0,
                                 fptr(gamma.detach()), fptr(beta.detach()), float(eps), N, HW, C, groups, ACT[act],
                                 fptr(scale), fptr(shift), fptr(mean), fptr(rstd), stream())
            ctx.save_for_backward(y, scale, shift, mean, rstd, gamma)
            ctx.meta = (groups, act)
            ctx.pbeta = beta
            return z
        chunks = lib.adr_nc_reduce_chunks(HW, _stats_rows(N, HW))
        part = torch.empty(N * chunks * 2 * C, dtype=torch.float32, device=dev)
        scale = torch.empty(N * C, dtype=torch.float32, device=dev)
        shift = torch.empty(N * C, dtype=torch.float32, device=dev)
        mean = torch.empty(N * groups, dtype=torch.float32, device=dev)
        rstd = torch.empty(N * groups, dtype=torch.float32, device=dev)
        lib.adr_nc_reduce(dcode(dtype), 0, ctypes.c_void_p(yp), ycs, 0, None, 0, 0, None, None, 0, 0, N, HW, C,
                          _stats_rows(N, HW), fptr(part), stream())
        lib.adr_gn_finalize(fptr(part), N, chunks, C, groups, float(HW * (C // groups)), fptr(gamma.detach()),
                            fptr(beta.detach()), float(eps), fptr(scale), fptr(shift), fptr(mean), fptr(rstd),
                            stream())
        z = empty_act(N, C, H, W, dtype, dev)
        lib.adr_affine_act(dcode(dtype), ctypes.c_void_p(yp), ycs, 0, ctypes.c_void_p(z.data_ptr()), C, 0,
                           fptr(scale), fptr(shift), 1, ACT[act], N, HW, C, stream())
        ctx.save_for_backward(y, scale, shift, mean, rstd, gamma)
        ctx.meta = (groups, act)
        ctx.pbeta = beta
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
        if ctx.fused:
            part = torch.empty(N * 2 * C, dtype=torch.float32, device=dev)
            dy = empty_act(N, C, H, W, y.dtype, dev)
            lib.adr_gn_act_bwd_fused(dt, ctypes.c_void_p(yp), ycs, 0, ctypes.c_void_p(dzp), dzcs, 0,
                                     ctypes.c_void_p(dy.data_ptr()), C, 0, fptr(scale), fptr(shift), fptr(mean),
                                     fptr(rstd), fptr(gamma.detach()), N, HW, C, groups, ACT[act], fptr(part),
                                     stream())
            dgamma, pg, acc_g = grad_dst(gamma, C, dev)
            dbeta, pb, acc_b = grad_dst(ctx.pbeta, C, dev)
            if acc_g != acc_b:
                raise RuntimeError("GN gamma/beta gradients must share one destination kind")
            if _defer_gn(acc_g):
                _dfr().add_gnparam(part, mean, rstd, pg, pb, N, 1, C, groups, acc_g)
            else:
                lib.adr_gn_param_grad(fptr(part), N, C, groups, fptr(mean), fptr(rstd), pg, pb, acc_g, stream())
            if ctx.gate is not None:
                _gn_gate_grad(ctx.gate, ctx.eps, part, [1], N, 1, HW, C, groups, [gamma.detach()], mean, rstd, dy)
            return dy, grad_ret(gamma, dgamma), grad_ret(ctx.pbeta, dbeta), None, None, None
        chunks = lib.adr_nc_reduce_chunks(HW, _stats_rows(N, HW))
        part = torch.empty(N * chunks * 2 * C, dtype=torch.float32, device=dev)
        dgamma, pg, acc_g = grad_dst(gamma, C, dev)
        dbeta, pb, acc_b = grad_dst(ctx.pbeta, C, dev)
        if acc_g != acc_b:
            raise RuntimeError("GN gamma/beta gradients must share one destination kind")
        A = torch.empty(N * C, dtype=torch.float32, device=dev)
        B = torch.empty(N * C, dtype=torch.float32, device=dev)
        Cc = torch.empty(N * C, dtype=torch.float32, device=dev)
        dfr = _defer_gn(acc_g)  # dgamma / dbeta at the flush, batched (the coefficients are needed now)
        if dfr:
            _dfr().add_gnparam(part, mean, rstd, pg, pb, N, chunks, C, groups, acc_g)
        lib.adr_nc_reduce(dt, 1, ctypes.c_void_p(yp), ycs, 0, ctypes.c_void_p(dzp), dzcs, 0, fptr(scale),
                          fptr(shift), 1, ACT[act], N, HW, C, _stats_rows(N, HW), fptr(part), stream())
        lib.adr_gn_bwd_finalize(fptr(part), N, chunks, C, groups, float(HW * (C // groups)), fptr(mean),
                                fptr(rstd), fptr(gamma.detach()), None if dfr else pg, None if dfr else pb,
                                fptr(A), fptr(B), fptr(Cc), acc_g, stream())
        dy = empty_act(N, C, H, W, y.dtype, dev)
        lib.adr_affine_act_bwd(dt, ctypes.c_void_p(yp), ycs, 0, ctypes.c_void_p(dzp), dzcs, 0,
                               ctypes.c_void_p(dy.data_ptr()), C, 0, fptr(scale), fptr(shift), fptr(A), fptr(B),
                               fptr(Cc), 1, 1, ACT[act], N, HW, C, 0, stream())
        if ctx.gate is not None:
            _gn_gate_grad(ctx.gate, ctx.eps, part, [1], N, chunks, HW, C, groups, [gamma.detach()], mean, rstd, dy)
        return dy, grad_ret(gamma, dgamma), grad_ret(ctx.pbeta, dbeta), None, None, None


class StemConvFn(torch.autograd.Function):
    """model.0 Conv(3, K, 3, 2)'s convolution read straight from the NCHW image batch (bf16 compute): fp32 images
    (already preprocessed), or the dataloader's uint8 batch with preprocess_batch's /255 (detect/train.py:57-59)
    applied inside the kernel. Returns the pre-BN output (NHWC bf16) and its BatchNorm partial statistics;
    backward = the weight gradient only (the image needs none)."""

    @staticmethod
    def forward(ctx, img, w, want_stats):
        ctx.set_materialize_grads(False)
        _req_cuda(img)
        u8 = img.dtype == torch.uint8
        img = img.contiguous() if u8 else img.float().contiguous()
        N, _, H, W = img.shape
        Kc = w.shape[0]
        Ho, Wo = (H - 1) // 2 + 1, (W - 1) // 2 + 1
        y = empty_act(N, Kc, Ho, Wo, torch.bfloat16, img.device)
        stats = None
        if want_stats:
            stats = torch.empty(lib.adr_stem_fwd_tiles(N, Ho) * 2 * Kc, dtype=torch.float32, device=img.device)
        wf = w.detach().float().contiguous()
        (lib.adr_stem_conv_fwd_u8 if u8 else lib.adr_stem_conv_fwd)(
            fptr(img), N, H, W, fptr(wf), Kc, ctypes.c_void_p(y.data_ptr()), Kc, fptr(stats), stream())
        ctx.save_for_backward(img)
        ctx.pw = w
        if stats is None:
            stats = torch.empty(0, device=img.device)
        ctx.mark_non_differentiable(stats)
        return y, stats

    @staticmethod
    def backward(ctx, dy, _dstats):
        if dy is None:
            return None, None, None
        (img,) = ctx.saved_tensors
        N, _, H, W = img.shape
        w = ctx.pw
        Kc = w.shape[0]
        dy, dyp, dycs = nhwc(dy.to(torch.bfloat16) if dy.dtype != torch.bfloat16 else dy)
        dw, pdw, acc = grad_dst(w, w.numel(), img.device)
        wsb = lib.adr_stem_wgrad_workspace(N, H, W, Kc)
        ws = torch.empty(wsb // 4 + 1, dtype=torch.float32, device=img.device)
        (lib.adr_stem_conv_wgrad_u8 if img.dtype == torch.uint8 else lib.adr_stem_conv_wgrad)(
            fptr(img), N, H, W, ctypes.c_void_p(dyp), dycs, Kc, pdw, acc, fptr(ws), wsb, stream())
        return None, grad_ret(w, dw), None


def stem_conv(img, w, want_stats):
    return StemConvFn.apply(img, w, want_stats)


def image_to_nhwc(img: torch.Tensor, dtype, cpad=8):
    """(B, 3, H, W) float images, or uint8 images (divided by 255 on the way, preprocess_batch) -> NHWC
    compute-dtype activation with channels padded to `cpad`."""
    _req_cuda(img)
    u8 = img.dtype == torch.uint8
    if not u8:
        img = img.float()
    if not img.is_contiguous():
        relayout_count[0] += 1
        img = img.contiguous()
    N, C, H, W = img.shape
    out = empty_act(N, cpad, H, W, dtype, img.device)
    (lib.adr_image_u8_to_nhwc if u8 else lib.adr_image_to_nhwc)(dcode(dtype), fptr(img),
                                                                ctypes.c_void_p(out.data_ptr()), N, C, H, W, cpad,
                                                                stream())
    return out


# ---------------------------------------------------------------------------------------------------------
# functional entry points
# ---------------------------------------------------------------------------------------------------------


def conv2d(x, w, b=None, stride=1, pad=0, want_stats=False, cpad=0, out=None):
    """y = conv2d(x, w) (+b); with `out` (an NHWC channel slice of a concat buffer) y is written into it."""
    y, stats = Conv2dFn.apply(x, w, b, stride, pad, want_stats, cpad, None if out is None else OutBox(out))
    return y, stats


# Training conv + bias + activation in one launch for the activations whose derivative follows from the output
# (relu, sigmoid: the AYHead gates and the cls_prob branch, head.py:135-136, 159-160, 269-270); ADR_CONV_ACT_FUSE=0
# runs the conv, then the activation kernel
CONV_ACT_FUSE = bool(int(__import__("os").environ.get("ADR_CONV_ACT_FUSE", "1")))
_ONES = {}


def _ones(n, dev):
    t = _ONES.get((n, dev))
    if t is None:
        t = _ONES[(n, dev)] = torch.ones(n, dtype=torch.float32, device=dev)
    return t


def conv_fwd_act(d, xp, wp, bf, K, act, yp):
    """act(conv + b) on the bf16 engine's epilogue (adr_conv2d_fwd_bf16_act with scale 1, shift = bias)."""
    dev = torch.device("cuda", torch.cuda.current_device())
    shift = bf if bf is not None else _zeros_f32(K, dev)
    sym = "" if _TIMING is None else _conv2_symbol(d, False).replace("conv_bf16_kernel", "conv_bf16_act_kernel")
    tok = _t0(sym, *_conv_work(d), _shape(d, "fwd+act") if _TIMING is not None else "")
    lib.adr_conv2d_fwd_bf16_act(ctypes.byref(d), ctypes.c_void_p(xp), ctypes.c_void_p(wp), fptr(_ones(K, dev)),
                                fptr(shift), ACT[act], ctypes.c_void_p(yp), stream())
    _t1(tok)


def _zeros_f32(n, dev):
    t = _ONES.get(("z", n, dev))
    if t is None:
        t = _ONES[("z", n, dev)] = torch.zeros(n, dtype=torch.float32, device=dev)
    return t


def conv_act(x, w, b, stride, pad, act, cpad=0):
    """act(conv2d(x, w) + b) for act in (relu, sigmoid); fused into the conv epilogue on the bf16 engine."""
    if CONV_ACT_FUSE and act in ("relu", "sigmoid") and x.dtype == torch.bfloat16:
        _, _, xcs = nhwc(x)
        N, C, H, W = x.shape
        K, Cw, R, S = w.shape
        (sh, sw), (ph, pw) = _pair(stride), _pair(pad)
        d, _, _ = conv_desc(N, H, W, C, xcs, K, R, S, sh, sw, ph, pw, K, x.dtype)
        if _engine2(d, d.c):
            y, _ = Conv2dFn.apply(x, w, b, stride, pad, False, cpad, None, act)
            return y
    return ActFn.apply(conv2d(x, w, b, stride, pad, False, cpad)[0], act)


def conv_transpose2d(x, w, b, stride, pad, out_pad):
    return ConvT2dFn.apply(x, w, b, stride, pad, out_pad)


class OutBox:
    """A caller-provided output view (a channel slice of a concat buffer) passed to a Function as a non-tensor
    argument, so autograd does not treat the destination as an input being modified in place."""
    __slots__ = ("t",)

    def __init__(self, t):
        self.t = t


def _out_view(box, N, C, H, W, dtype, dev):
    """(tensor, ptr, channel stride) of the output: the boxed view, or a fresh NHWC activation."""
    if box is None:
        z = empty_act(N, C, H, W, dtype, dev)
        return z, z.data_ptr(), C
    z = box.t
    if tuple(z.shape) != (N, C, H, W) or z.dtype != dtype:
        raise RuntimeError(f"out view {tuple(z.shape)} {z.dtype} != {(N, C, H, W)} {dtype}")
    z, ptr, cs = nhwc(z)
    if z is not box.t:
        raise RuntimeError("out view is not an NHWC channel slice")
    return z, ptr, cs


def _bn_eval_coefs_into(bn, scale, shift):
    C = scale.numel()
    lib.adr_bn_finalize(None, 0, C, 1.0, fptr(bn.weight.detach()), fptr(bn.bias.detach()), fptr(bn.running_mean),
                        fptr(bn.running_var), float(bn.momentum), float(bn.eps), 0, fptr(scale), fptr(shift), None,
                        None, stream())


def _bn_eval_coefs(bn, dev):
    """(scale, shift) of BatchNorm2d with running statistics (one adr_bn_finalize launch, or the predictor's
    cached pair)."""
    pc = _PACK
    if pc is not None and pc.cache_bn_coefs:
        hit = pc.bn_coefs.get(id(bn))
        if hit is not None and hit[0] is bn:
            return hit[1], hit[2]
    C = bn.num_features
    scale = torch.empty(C, dtype=torch.float32, device=dev)
    shift = torch.empty(C, dtype=torch.float32, device=dev)
    _bn_eval_coefs_into(bn, scale, shift)
    if pc is not None and pc.cache_bn_coefs:
        pc.bn_coefs[id(bn)] = (bn, scale, shift)
    return scale, shift


EVAL_CONV_BN_ACT = bool(int(__import__("os").environ.get("ADR_EVAL_FUSE", "1")))  # 0: conv, then BN + act


def conv_bn_act_eval(x, w, stride, pad, bn, act: str, cpad=0, out=None):
    """Inference Conv-BN-act (no autograd): act(BN_eval(conv2d(x, w))) in ONE bf16-engine launch — the BatchNorm
    affine and the activation run on the fp32 accumulator in the conv epilogue (adr_conv2d_fwd_bf16_act), as the
    reference predictor runs Conv.forward_fuse after fuse_conv_and_bn (nn/modules/conv.py:52-54,
    nn/tasks.py:203-218). Returns None when the contraction is not on the bf16 engine (the caller then runs the
    unfused pair)."""
    dtype = x.dtype
    if dtype != torch.bfloat16 or torch.is_grad_enabled():
        return None
    x, xp, xcs = nhwc(x)
    N, C, H, W = x.shape
    K, Cw, R, S = w.shape
    Cp = max(Cw, cpad)
    if C != Cp:
        raise RuntimeError(f"conv_bn_act_eval: input has {C} channels, weight expects {Cw} (padded {Cp})")
    (sh, sw), (ph, pw) = _pair(stride), _pair(pad)
    Ho, Wo = (H + 2 * ph - R) // sh + 1, (W + 2 * pw - S) // sw + 1
    y, yp, ycs = _out_view(None if out is None else OutBox(out), N, K, Ho, Wo, dtype, x.device)
    d, Ho, Wo = conv_desc(N, H, W, C, xcs, K, R, S, sh, sw, ph, pw, ycs, dtype)
    if not _engine2(d, d.c) or (CONV_FP8 and C >= _FP8_MIN_C and R * S > 1):
        return None
    wp, _ = pack_weight2(w, dtype, cpad)
    scale, shift = _bn_eval_coefs(bn, x.device)
    sym = "" if _TIMING is None else _conv2_symbol(d, False).replace("conv_bf16_kernel", "conv_bf16_act_kernel")
    tok = _t0(sym, *_conv_work(d), _shape(d, "fwd+bn+act") if _TIMING is not None else "")
    lib.adr_conv2d_fwd_bf16_act(ctypes.byref(d), ctypes.c_void_p(xp), ctypes.c_void_p(wp.data_ptr()), fptr(scale),
                                fptr(shift), ACT[act], ctypes.c_void_p(yp), stream())
    _t1(tok)
    return y if out is None else out


def bn_act(y, stats, bn: torch.nn.Module, act: str, training: bool, out=None, xfuse=False, lazy=False, res=None):
    """act(BatchNorm(y)) (+ res). xfuse: y is a dense conv's output read only here (Conv.forward), so the backward may
    hand its dy to that conv's data gradient unwritten (BnXf). lazy: the caller's consumer is a conv that can stage y
    through the BN-act itself (BnFwd). res: a residual added in the same pass (adr_affine_act_res)."""
    return BNActFn.apply(y, stats, bn.weight, bn.bias, bn.running_mean, bn.running_var, act, training, bn.momentum,
                         bn.eps, None if out is None else OutBox(out), xfuse, lazy and res is None, res)


def gn_act(y, gn: torch.nn.Module, act: str):
    return GNActFn.apply(y, gn.weight, gn.bias, gn.num_groups, act, gn.eps)


# ---------------------------------------------------------------------------------------------------------
# elementwise glue
# ---------------------------------------------------------------------------------------------------------
EW_COPY, EW_AXPBY, EW_MUL, EW_FMA, EW_ACT, EW_ACT_BWD, EW_ADD3, EW_ACT_BWD_OUT, EW_MUL_ADD = range(9)


_CONSTS = {}


def _const(value, device):
    """A cached 1-element fp32 device tensor (kernel scalar operands; no fill launch per use)."""
    key = (float(value), str(device))
    t = _CONSTS.get(key)
    if t is None:
        t = _CONSTS[key] = torch.full((1,), float(value), dtype=torch.float32, device=device)
    return t


def _ew(op, out, a, b=None, c=None, act=0, ca=None, cb=None, accumulate=0):
    """Launch adr_ew over same-shaped NHWC views (a, b, c, out are (tensor, ptr, cs) triples or None)."""
    t = a[0]
    N, C, H, W = t.shape
    lib.adr_ew(dcode(t.dtype), op, act, ctypes.c_void_p(a[1]), a[2], ctypes.c_void_p(b[1]) if b else None,
               b[2] if b else 0, ctypes.c_void_p(c[1]) if c else None, c[2] if c else 0, ctypes.c_void_p(out[1]),
               out[2], N * H * W, C, fptr(ca), fptr(cb), accumulate, stream())


def _v(t):
    return nhwc(t)


def _new_like(t):
    n, c, h, w = t.shape
    return empty_act(n, c, h, w, t.dtype, t.device)


class CatFn(torch.autograd.Function):
    """torch.cat(xs, dim=1) on NHWC: one copy per piece into the concat buffer; backward = zero-copy slices."""

    @staticmethod
    def forward(ctx, box, *xs):
        t0 = xs[0]
        N, _, H, W = t0.shape
        Ctot = sum(x.shape[1] for x in xs)
        out = empty_act(N, Ctot, H, W, t0.dtype, t0.device) if box is None else box.t
        if tuple(out.shape) != (N, Ctot, H, W) or out.stride(1) != 1 or out.stride(3) != Ctot:
            raise RuntimeError("cat: out buffer must be a whole NHWC activation of the concat shape")
        off = 0
        sizes, todo = [], []
        for x in xs:
            v = _v(x)
            o = out[:, off:off + x.shape[1]]
            if not (v[1] == o.data_ptr() and v[2] == Ctot):  # producers that wrote in place need no copy
                todo.append((o, v, x.shape[1]))
            sizes.append(x.shape[1])
            off += x.shape[1]
        if len(todo) > 1 and _TIMING is None and t0.dtype == torch.bfloat16 and all(
                c % 8 == 0 and v[2] % 8 == 0 and v[1] % 16 == 0 and o.data_ptr() % 16 == 0 for o, v, c in todo):
            # every piece that needs a copy in one launch (adr_copy_pieces; bitwise the per-piece copies)
            arr = (CopyPiece * len(todo))(*[CopyPiece(v[1], o.data_ptr(), v[2], Ctot, c, 0) for o, v, c in todo])
            lib.adr_copy_pieces(ctypes.cast(arr, ctypes.c_void_p), len(todo), N * H * W, stream())
        else:
            for o, v, _ in todo:
                _ew(EW_COPY, (o, o.data_ptr(), Ctot), v)
        ctx.sizes = sizes
        # pieces that are fan-out views with a gradient sink: backward can make their slice the sink's buffer
        ctx.sinks = [getattr(x, "_adr_sink", None) for x in xs]
        return out if box is None else out[:, :]

    @staticmethod
    def backward(ctx, dy):
        dy, _, _ = _v(dy)
        outs, off = [], 0
        for s, sk in zip(ctx.sizes, ctx.sinks):
            piece = dy[:, off:off + s]
            piece._adr_excl = True  # a disjoint slice handed to exactly one consumer: FanOutFn may add into it
            # a fan-out view whose conv consumers have not run backward yet: they accumulate into the slice
            outs.append(None if sk is not None and sk.seed(piece) else piece)
            off += s
        return (None,) + tuple(outs)


def cat(xs, out=None):
    """torch.cat(xs, 1). With `out` (an NHWC concat buffer whose slices some producers already wrote through
    their own `out=` views), only the pieces that are not in place are copied."""
    return CatFn.apply(None if out is None else OutBox(out), *xs)


def zero_(t):
    """Zero a device tensor's storage span with hipMemsetAsync (via libadr)."""
    lib.adr_memset_zero(ctypes.c_void_p(t.data_ptr()), t.numel() * t.element_size(), stream())
    return t


class SplitFn(torch.autograd.Function):
    """x.split(sizes, dim=1) as zero-copy NHWC views; backward assembles the piece gradients into one NHWC
    gradient buffer with libadr copies (absent pieces are zero-filled), keeping grads channels_last."""

    @staticmethod
    def forward(ctx, x, sizes):
        ctx.set_materialize_grads(False)
        ctx.meta = (tuple(sizes), x.shape, x.dtype)
        outs, off = [], 0
        for sz in sizes:
            outs.append(x[:, off:off + sz])
            off += sz
        return tuple(outs)

    @staticmethod
    def backward(ctx, *grads):
        sizes, shape, dtype = ctx.meta
        N, C, H, W = shape
        joined = _adjacent_slices(grads, sizes, dtype)
        if joined is not None:  # the pieces are consecutive channel slices of one buffer (a concat gradient)
            return joined, None
        dev = next(g for g in grads if g is not None).device
        dx = empty_act(N, C, H, W, dtype, dev)
        off = 0
        for g, sz in zip(grads, sizes):
            piece = dx[:, off:off + sz]
            if g is None:
                # zero the slice: o = 0*piece + 0*piece would read garbage; copy from a zero tensor instead
                z = zero_(empty_act(N, sz, H, W, dtype, dev))
                _ew(EW_COPY, (piece, piece.data_ptr(), C), _v(z))
            else:
                _ew(EW_COPY, (piece, piece.data_ptr(), C), _v(g.to(dtype) if g.dtype != dtype else g))
            off += sz
        return dx, None


def split(x, sizes):
    return SplitFn.apply(x, list(sizes))


def _adjacent_slices(grads, sizes, dtype):
    """One NHWC view spanning `grads` when they are consecutive channel slices of one buffer, else None."""
    if any(g is None or g.dtype != dtype for g in grads):
        return None
    g0 = grads[0]
    cs, es, st = g0.stride(3), g0.element_size(), g0.untyped_storage().data_ptr()
    off = 0
    for g, sz in zip(grads, sizes):
        if g.shape[1] != sz or g.stride() != g0.stride() or g.untyped_storage().data_ptr() != st or \
                g.data_ptr() != g0.data_ptr() + off * es or (g.stride(1) != 1 and sz > 1):
            return None
        off += sz
    if off > cs:
        return None
    n, _, h, w = g0.shape
    return torch.as_strided(g0, (n, off, h, w), g0.stride(), g0.storage_offset())


class GradSink:
    """Gradient destination shared by the views of one FanOutFn: a consumer whose backward can accumulate in its
    epilogue (Conv2dFn's dgrad) writes its input gradient here — the first one plainly, later ones accumulating —
    and hands autograd None, so FanOutFn sums one gradient fewer (per conv consumer: a 2-read + 1-write pass and a
    launch become one extra read in the dgrad epilogue). Single stream, so the order is autograd's."""
    __slots__ = ("buf", "shape", "dtype", "pend", "site")

    def __init__(self, shape, dtype):
        self.buf, self.shape, self.dtype, self.site = None, tuple(shape), dtype, None
        self.pend = []  # pass-through gradients (AddFn's) waiting to be folded into a conv consumer's dgrad

    @staticmethod
    def _aligned(t):
        n, c, h, w = t.shape
        s0, s1, s2, s3 = t.stride()
        return s1 == 1 and s2 == w * s3 and s0 == h * w * s3 and t.data_ptr() % 16 == 0 and s3 % 8 == 0

    def defer(self, g):
        """Hold a pass-through gradient (a residual add hands its output gradient unchanged to this input): the next
        conv consumer to claim the buffer adds it in its dgrad epilogue, FanOutFn adds whatever is left. bf16 only
        (the bf16 engine's epilogue); `g` is marked so FanOutFn never accumulates into it in place."""
        if not _DEFER_ADD or g is None or not self.fits(g) or g.dtype != torch.bfloat16 or not self._aligned(g):
            return False
        g._adr_pinned = True
        self.pend.append(g)
        return True

    def fits(self, t):
        return t is not None and tuple(t.shape) == self.shape and t.dtype == self.dtype

    def seed(self, piece):
        """Make an exclusive concat-gradient slice (CatFn.backward) the shared buffer before any conv consumer
        has claimed one: the convs then accumulate straight into it and FanOutFn gets one gradient fewer to add
        (the acc += sink pass). False when a consumer already claimed a buffer or the slice is not an aligned NHWC
        view the dgrad epilogue can write."""
        if self.buf is not None or not self.fits(piece) or not _SEED_CAT or not self._aligned(piece):
            return False
        self.buf = piece
        return True

    def claim(self, device, can_add=False):
        """(NHWC gradient buffer, accumulate flag, addend or None) for the next consumer; with can_add the
        consumer takes one pending pass-through gradient into its epilogue."""
        add = self.pend.pop(0) if can_add and self.pend else None
        if self.buf is None:
            N, C, H, W = self.shape
            self.buf = empty_act(N, C, H, W, self.dtype, device)
            return self.buf, 0, add
        return self.buf, 1, add


def _sink_of(x):
    """The fan-out gradient sink of x when a consumer's backward can write / accumulate x's gradient into it."""
    sk = getattr(x, "_adr_sink", None)
    # the shared buffer must be a vector-aligned NHWC tensor (nhwc() would otherwise hand out a relaid copy)
    return sk if sk is not None and sk.fits(x) and x.shape[1] % (16 // x.element_size()) == 0 else None


def _defer_pass(sk, dy):
    """A pass-through input gradient (res / base / addend: the op hands dy on unchanged): held in the input's
    fan-out sink for a conv consumer's dgrad epilogue when possible (GradSink.defer); else dy for autograd."""
    return None if sk is not None and sk.defer(dy) else dy


def _dx_dst(ctx, shape, dtype, dev):
    """(buffer, accumulate) for a consumer's input gradient: the fan-out sink's shared buffer (claimed; the
    consumer returns None to autograd) or a fresh NHWC tensor."""
    if ctx.sink is not None:
        buf, acc, _ = ctx.sink.claim(dev)
        return buf, acc
    return empty_act(*shape, dtype, dev), 0


FANOUT_LOG = None  # a list: FanOutFn.backward records (creation site, autograd grads, sink buf, seeded, pending)
_FANOUT_SINK = bool(int(__import__("os").environ.get("ADR_FANOUT_SINK", "1")))
_SEED_CAT = bool(int(__import__("os").environ.get("ADR_SEED_CAT", "1")))  # 0: CatFn hands every slice to autograd
_SHARE_SINK = bool(int(__import__("os").environ.get("ADR_SHARE_SINK", "1")))  # 0: every fan-out owns a sink
_DEFER_ADD = bool(int(__import__("os").environ.get("ADR_DEFER_ADD", "1")))  # 0: AddFn returns its gradient as is


class FanOutFn(torch.autograd.Function):
    """x used by n consumers, as n views. Backward sums the n gradients with HIP launches (one for 2 or 3 of
    them) — into one that is an exclusive concat-gradient slice when there is one (no new buffer, and the split
    that produced x can then hand its gradient back as a view) — instead of autograd's own accumulation, which
    is one PyTorch add per extra consumer (a slow strided kernel on channel slices)."""

    @staticmethod
    def forward(ctx, x, n, sink):
        ctx.set_materialize_grads(False)
        ctx.sink = sink
        return tuple(x[:, :] for _ in range(n))

    @staticmethod
    def backward(ctx, *grads):
        gs = [g for g in grads if g is not None]
        sink = ctx.sink
        if FANOUT_LOG is not None:  # diagnostics (scripts/ew_sites.py): what each fan-out still sums here
            FANOUT_LOG.append((sink.site if sink is not None else "?", len(gs),
                               sink is not None and sink.buf is not None,
                               sink is not None and sink.buf is not None and getattr(sink.buf, "_adr_excl", False),
                               len(sink.pend) if sink is not None else 0, tuple(gs[0].shape) if gs else None))
        if sink is not None and sink.buf is not None:  # the consumers that accumulated into the shared buffer
            # a seeded concat slice (GradSink.seed) goes first: it is the accumulation target below, so x's
            # gradient stays that slice (SplitFn can then join it with its neighbours without a copy)
            if getattr(sink.buf, "_adr_excl", False):
                gs.insert(0, sink.buf)
            else:
                gs.append(sink.buf)
            sink.buf = None
        if sink is not None and sink.pend:  # pass-through gradients no conv consumer took
            gs.extend(sink.pend)
            sink.pend = []
        if not gs:
            return None, None, None
        if len(gs) == 1:
            if _DEBUG_BNSTAT:
                gs[0]._adr_src = "fanout(1)"
            return gs[0], None, None
        dt = gs[0].dtype
        gs = [g if g.dtype == dt else g.to(dt) for g in gs]
        excl = [g for g in gs if getattr(g, "_adr_excl", False) and not getattr(g, "_adr_pinned", False)
                and _v(g)[0] is g]
        if excl:  # accumulate the others into the exclusive slice in place
            acc = excl[0]
            rest = [g for g in gs if g is not acc]
            va = _v(acc)
            while rest:
                if len(rest) >= 2:
                    _ew(EW_AXPBY, va, _v(rest[0]), _v(rest[1]), accumulate=1)  # acc += r0 + r1
                    rest = rest[2:]
                else:
                    _ew(EW_COPY, va, _v(rest[0]), accumulate=1)
                    rest = rest[1:]
            if _DEBUG_BNSTAT:
                acc._adr_src = f"fanout-excl({len(gs)})"
            return acc, None, None
        out = _new_like(_v(gs[0])[0])
        vo = (out, out.data_ptr(), out.shape[1])
        if len(gs) >= 3:
            _ew(EW_ADD3, vo, _v(gs[0]), _v(gs[1]), _v(gs[2]))
            rest = gs[3:]
        else:
            _ew(EW_AXPBY, vo, _v(gs[0]), _v(gs[1]))
            rest = []
        while rest:
            if len(rest) >= 2:
                _ew(EW_AXPBY, vo, _v(rest[0]), _v(rest[1]), accumulate=1)
                rest = rest[2:]
            else:
                _ew(EW_COPY, vo, _v(rest[0]), accumulate=1)
                rest = rest[1:]
        if _DEBUG_BNSTAT:
            out._adr_src = f"fanout({len(gs)})"
        return out, None, None


def fanout(x, n=2):
    """n views of x whose gradients are summed by libadr (see FanOutFn); conv consumers deliver theirs through a
    shared GradSink."""
    # a fan-out of a fan-out view (a block that fans out its input, fed from an outer fan-out) shares the outer
    # sink: consumers on both levels accumulate into one buffer (often the outer's seeded concat slice), so
    # neither FanOutFn has a sum left to launch; each gradient still reaches the outer sum exactly once
    outer = _sink_of(x) if _SHARE_SINK else None
    sink = outer if outer is not None else (GradSink(x.shape, x.dtype) if _FANOUT_SINK else None)
    if sink is not None and outer is None and FANOUT_LOG is not None:
        import sys
        f = sys._getframe(1)
        while f is not None and f.f_code.co_filename == __file__:
            f = f.f_back
        if f is not None:
            sink.site = f"{f.f_code.co_filename.rsplit('/', 1)[-1]}:{f.f_lineno}:{f.f_code.co_name}"
    outs = FanOutFn.apply(x, n, sink)
    if sink is not None:
        for o in outs:
            o._adr_sink = sink
    return outs


class AddFn(torch.autograd.Function):
    """a + b (+ c)."""

    @staticmethod
    def forward(ctx, a, b, c=None, box=None):
        va, vb = _v(a), _v(b)
        N, C, H, W = va[0].shape
        o = _out_view(box, N, C, H, W, va[0].dtype, va[0].device)
        if c is None:
            _ew(EW_AXPBY, o, va, vb)
        else:
            _ew(EW_ADD3, o, va, vb, _v(c))
        ctx.three = c is not None
        # inputs that are fan-out views with a gradient sink: backward defers its pass-through gradient there
        ctx.sinks = [getattr(t, "_adr_sink", None) for t in (a, b, c)]
        return o[0]

    @staticmethod
    def backward(ctx, dy):
        outs = [dy, dy, dy if ctx.three else None]
        for i, sk in enumerate(ctx.sinks):
            if outs[i] is not None and sk is not None and sk.defer(dy):
                outs[i] = None  # a conv consumer of that fan-out adds dy in its dgrad epilogue
        return outs[0], outs[1], outs[2], None


def add(a, b, c=None, out=None):
    return AddFn.apply(a, b, c, None if out is None else OutBox(out))


class MulFn(torch.autograd.Function):
    """a * b (Multiply, block.py:1442-1447)."""

    @staticmethod
    def forward(ctx, a, b):
        va, vb = _v(a), _v(b)
        out = _new_like(va[0])
        _ew(EW_MUL, (out, out.data_ptr(), out.shape[1]), va, vb)
        ctx.save_for_backward(va[0], vb[0])
        return out

    @staticmethod
    def backward(ctx, dy):
        a, b = ctx.saved_tensors
        vd = _v(dy)
        da = db = None
        if ctx.needs_input_grad[0]:
            da = _new_like(a)
            _ew(EW_MUL, (da, da.data_ptr(), da.shape[1]), vd, _v(b))
        if ctx.needs_input_grad[1]:
            db = _new_like(b)
            _ew(EW_MUL, (db, db.data_ptr(), db.shape[1]), vd, _v(a))
        return da, db


def mul(a, b):
    return MulFn.apply(a, b)


class MulAddFn(torch.autograd.Function):
    """Add(Multiply(p, q), r) (block.py:1442-1453, the HS-FPN gate and its residual) in one pass (EW_MUL_ADD: the
    product rounded to the compute dtype before the add); forward and backward bitwise MulFn + AddFn."""

    @staticmethod
    def forward(ctx, p, q, r):
        vp, vq, vr = _v(p), _v(q), _v(r)
        out = _new_like(vp[0])
        _ew(EW_MUL_ADD, (out, out.data_ptr(), out.shape[1]), vp, vq, vr)
        ctx.save_for_backward(vp[0], vq[0])
        ctx.sr = getattr(r, "_adr_sink", None)
        return out

    @staticmethod
    def backward(ctx, dy):
        p, q = ctx.saved_tensors
        vd = _v(dy)
        dp = dq = None
        if ctx.needs_input_grad[0]:
            dp = _new_like(p)
            _ew(EW_MUL, (dp, dp.data_ptr(), dp.shape[1]), vd, _v(q))
        if ctx.needs_input_grad[1]:
            dq = _new_like(q)
            _ew(EW_MUL, (dq, dq.data_ptr(), dq.shape[1]), vd, _v(p))
        return dp, dq, (_defer_pass(ctx.sr, dy) if ctx.needs_input_grad[2] else None)


def mul_add(p, q, r):
    return MulAddFn.apply(p, q, r)


class FmaFn(torch.autograd.Function):
    """a + b * c (gated residual, CrossTaskInteraction head.py:744-745)."""

    @staticmethod
    def forward(ctx, a, b, c):
        va, vb, vc = _v(a), _v(b), _v(c)
        out = _new_like(va[0])
        _ew(EW_FMA, (out, out.data_ptr(), out.shape[1]), va, vb, vc)
        ctx.save_for_backward(vb[0], vc[0])
        ctx.sa, ctx.sink = getattr(a, "_adr_sink", None), _sink_of(b)  # fan-out sinks: a's pass-through, b's product
        return out

    @staticmethod
    def backward(ctx, dy):
        b, c = ctx.saved_tensors
        vd = _v(dy)
        db, acc = _dx_dst(ctx, tuple(b.shape), b.dtype, b.device)
        _ew(EW_MUL, _v(db), vd, _v(c), accumulate=acc)
        dc = _new_like(c)
        _ew(EW_MUL, (dc, dc.data_ptr(), dc.shape[1]), vd, _v(b))
        return _defer_pass(ctx.sa, dy), (None if ctx.sink is not None else db), dc


def fma(a, b, c):
    return FmaFn.apply(a, b, c)


class ActFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, act):
        vx = _v(x)
        out = _new_like(vx[0])
        _ew(EW_ACT, (out, out.data_ptr(), out.shape[1]), vx, act=ACT[act])
        ctx.save_for_backward(vx[0])
        ctx.act = act
        ctx.sink = _sink_of(x)
        return out

    @staticmethod
    def backward(ctx, dy):
        (x,) = ctx.saved_tensors
        dx, acc = _dx_dst(ctx, tuple(x.shape), x.dtype, x.device)
        _ew(EW_ACT_BWD, (dx, dx.data_ptr(), dx.stride(3)), _v(x), _v(dy), act=ACT[ctx.act], accumulate=acc)
        return (None if ctx.sink is not None else dx), None


def act(x, name):
    return x if name == "none" else ActFn.apply(x, name)


def _reduce_dot(x, dy, sum_n, sum_c, which=0):
    """sum over pixels of x*dy (which=0) or dy (which=1), per (n, c), optionally collapsed over n / c."""
    N, C, H, W = dy.shape
    vd = _v(dy)
    vx = _v(x) if x is not None else (None, 0, 0)
    chunks = lib.adr_nc_reduce_chunks(H * W, _stats_rows(N, H * W))
    part = torch.empty(N * chunks * 2 * C, dtype=torch.float32, device=dy.device)
    lib.adr_dot_reduce(dcode(dy.dtype), ctypes.c_void_p(vx[1]) if x is not None else None, vx[2],
                       ctypes.c_void_p(vd[1]), vd[2], N, H * W, C, _stats_rows(N, H * W), fptr(part), stream())
    out = torch.empty((1 if sum_n else N) * (1 if sum_c else C), dtype=torch.float32, device=dy.device)
    lib.adr_nc_collapse(fptr(part), N, chunks, C, which, fptr(out), int(sum_n), int(sum_c), 0, stream())
    return out


class ScaleFn(torch.autograd.Function):
    """x * g (+ res) with g a device tensor broadcast as: 'scalar' (shape ()), 'n' (N,), 'c' (C,), 'nc' (N, C)."""

    @staticmethod
    def forward(ctx, x, g, res, mode, box=None, from_out=False):
        vx = _v(x)
        N, C, H, W = x.shape
        gs = g.detach().float().contiguous()
        gns, gcs = {"scalar": (0, 0), "n": (1, 0), "c": (0, 1), "nc": (C, 1)}[mode]
        out, op, ocs = _out_view(box, N, C, H, W, x.dtype, x.device)
        vr = _v(res) if res is not None else None
        lib.adr_bcast_mul(dcode(x.dtype), ctypes.c_void_p(vx[1]), vx[2], fptr(gs), gns, gcs,
                          ctypes.c_void_p(vr[1]) if vr else None, vr[2] if vr else 0, ctypes.c_void_p(op),
                          ocs, N, H * W, C, 0, stream())
        # from_out (bf16, per-image gates feeding a normalisation): dg = sum(dy * out) / g from the very tensor the
        # next op consumed, instead of sum(dy * x) from the separately rounded x
        ctx.from_out = from_out and mode == "n" and res is None and x.dtype == torch.bfloat16
        ctx.save_for_backward(out if ctx.from_out else vx[0], gs)
        if ctx.from_out and box is None:
            out._adr_gate = gs  # the GroupNorm that reads out computes dL/dgs from its fp32 statistics
        ctx.meta = (mode, g.shape, res is not None)
        ctx.pg = g
        ctx.sink, ctx.sres = _sink_of(x), (getattr(res, "_adr_sink", None) if res is not None else None)
        return out if box is None else out[:, :]

    @staticmethod
    def backward(ctx, dy):
        x, gs = ctx.saved_tensors
        mode, gshape, has_res = ctx.meta
        N, C, H, W = x.shape
        vd = _v(dy)
        dx = dg = None
        if ctx.needs_input_grad[0]:
            dx, acc = _dx_dst(ctx, (N, C, H, W), x.dtype, x.device)
            vo = _v(dx)
            gns, gcs = {"scalar": (0, 0), "n": (1, 0), "c": (0, 1), "nc": (C, 1)}[mode]
            lib.adr_bcast_mul(dcode(x.dtype), ctypes.c_void_p(vd[1]), vd[2], fptr(gs), gns, gcs, None, 0,
                              ctypes.c_void_p(vo[1]), vo[2], N, H * W, C, acc, stream())
            if ctx.sink is not None:
                dx = None
        if ctx.needs_input_grad[1]:
            sum_n = mode in ("scalar", "c")
            sum_c = mode in ("scalar", "n")
            if sum_n and sum_c and _defer_dot(ctx.pg, x, vd[0]):  # a scalar: sum(x * dy) at the flush
                out = torch.empty(1, dtype=torch.float32, device=x.device)
                _dfr().add_dotsum(x, vd[0], out)
                dg = sink(ctx.pg, out.view(gshape))
            elif ctx.from_out:
                ent = _GATE_GRAD.pop(dy.data_ptr(), None)
                src = ent[0]() if ent is not None else None
                if src is not None and src.shape == dy.shape and \
                        src.untyped_storage().data_ptr() == dy.untyped_storage().data_ptr():
                    dg = sink(ctx.pg, ent[1].view(gshape))  # the GN backward's exact residue (adr_gn_gate_grad)
                else:
                    dg = sink(ctx.pg, (_reduce_dot(x, vd[0], sum_n, sum_c) / gs.clamp_min(1e-30)).view(gshape))
            else:
                dg = sink(ctx.pg, _reduce_dot(x, vd[0], sum_n, sum_c).view(gshape))
        return dx, dg, (_defer_pass(ctx.sres, dy) if has_res else None), None, None, None


def scale(x, g, mode, res=None, out=None, grad_from_out=False):
    """x * g broadcast by `mode`. grad_from_out: the gate gradient of a per-image gate ('n') is taken from the
    output (sum(dy * out) / g) — used where a normalisation follows, whose input gradient is orthogonal to the
    output it normalised, so the near-zero true gate gradient is not buried under the rounding of x (bf16)."""
    return ScaleFn.apply(x, g, res, mode, None if out is None else OutBox(out), grad_from_out)


class WeightedSumFn(torch.autograd.Function):
    """sum_i w[i] * x_i (+ base) with w a learnable device vector (PFF stage_attention, block.py:2626-2628)."""

    @staticmethod
    def forward(ctx, w, base, *xs):
        wd = w.detach().float().contiguous()
        out = _new_like(xs[0])
        vo = (out, out.data_ptr(), out.shape[1])
        # o = w0*x0 + (base or 0)*1 ; then o += w_i * x_i
        v0 = _v(xs[0])
        if base is not None:
            _ew(EW_AXPBY, vo, v0, _v(base), ca=wd[0:1])
        else:
            _ew(EW_AXPBY, vo, v0, v0, ca=wd[0:1], cb=_const(0.0, w.device))
        for i in range(1, len(xs)):
            vi = _v(xs[i])
            _ew(EW_AXPBY, vo, vi, vi, ca=wd[i:i + 1], cb=_const(0.0, w.device), accumulate=1)
        ctx.save_for_backward(wd, *[_v(x)[0] for x in xs])
        ctx.has_base = base is not None
        ctx.pw = w
        # fan-out sinks: each x_i's scaled gradient is written (accumulated) into its sink; base's passes through
        ctx.sinks = [_sink_of(x) for x in xs]
        ctx.sbase = getattr(base, "_adr_sink", None) if base is not None else None
        return out

    @staticmethod
    def backward(ctx, dy):
        wd, *xs = ctx.saved_tensors
        vd = _v(dy)
        dxs = []
        for i, (x, sk) in enumerate(zip(xs, ctx.sinks)):
            d, acc = sk.claim(dy.device)[:2] if sk is not None else (_new_like(x), 0)
            _ew(EW_AXPBY, _v(d), vd, vd, ca=wd[i:i + 1], cb=_const(0.0, dy.device), accumulate=acc)
            dxs.append(None if sk is not None else d)
        if not ctx.needs_input_grad[0]:
            dw = None
        elif all(_defer_dot(ctx.pw, x, vd[0]) for x in xs):  # the weights' scalar gradients at the flush
            dw = torch.empty(len(xs), dtype=torch.float32, device=dy.device)
            for i, x in enumerate(xs):
                _dfr().add_dotsum(x, vd[0], dw[i:i + 1])
        else:
            dw = torch.cat([_reduce_dot(x, vd[0], True, True) for x in xs])
        return (sink(ctx.pw, dw), _defer_pass(ctx.sbase, dy) if ctx.has_base else None, *dxs)


def weighted_sum(w, xs, base=None):
    return WeightedSumFn.apply(w, base, *xs)


class FusionFn(torch.autograd.Function):
    """Fusion('bifpn'): w = relu(fw)/(sum+1e-4); out = sum_i w_i x_i (block.py:1532-1535)."""

    @staticmethod
    def forward(ctx, fw, *xs):
        fwd = fw.detach().float().contiguous()
        w = torch.empty_like(fwd)
        lib.adr_fusion_weights(fptr(fwd), fwd.numel(), 1e-4, fptr(w), stream())
        out = _new_like(xs[0])
        vo = (out, out.data_ptr(), out.shape[1])
        v = [_v(x) for x in xs]
        _ew(EW_AXPBY, vo, v[0], v[1], ca=w[0:1], cb=w[1:2])
        for i in range(2, len(xs)):
            _ew(EW_AXPBY, vo, v[i], v[i], ca=w[i:i + 1], cb=_const(0.0, fw.device), accumulate=1)
        ctx.save_for_backward(fwd, w, *[t[0] for t in v])
        ctx.pfw = fw
        return out

    @staticmethod
    def backward(ctx, dy):
        fwd, w, *xs = ctx.saved_tensors
        vd = _v(dy)
        z = _const(0.0, dy.device)
        dxs = []
        for i, x in enumerate(xs):
            d = _new_like(x)
            _ew(EW_AXPBY, (d, d.data_ptr(), d.shape[1]), vd, vd, ca=w[i:i + 1], cb=z)
            dxs.append(d)
        dfw = torch.empty_like(fwd)
        if ctx.needs_input_grad[0] and all(_defer_dot(ctx.pfw, x, vd[0]) for x in xs):
            # the per-input dot sums at the flush (one batched launch with the other scalar gradients), then the
            # normalisation backward, then the arena add (the flush runs dots -> post_dots -> axpys)
            dwn = torch.empty(len(xs), dtype=torch.float32, device=dy.device)
            for i, x in enumerate(xs):
                _dfr().add_dotsum(x, vd[0], dwn[i:i + 1])
            n = fwd.numel()
            _dfr().post_dots.append(lambda: lib.adr_fusion_weights_bwd(fptr(fwd), n, 1e-4, fptr(dwn), fptr(dfw),
                                                                       stream()))
        else:
            dwn = torch.cat([_reduce_dot(x, vd[0], True, True) for x in xs])
            lib.adr_fusion_weights_bwd(fptr(fwd), fwd.numel(), 1e-4, fptr(dwn), fptr(dfw), stream())
        return (sink(ctx.pfw, dfw), *dxs)


def fusion(fw, xs):
    return FusionFn.apply(fw, *xs)


# ---------------------------------------------------------------------------------------------------------
# pooling
# ---------------------------------------------------------------------------------------------------------


class MaxPoolFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, k, box=None):
        vx = _v(x)
        N, C, H, W = x.shape
        y, yp, ycs = _out_view(box, N, C, H, W, x.dtype, x.device)
        arg = torch.empty(N * H * W * C, dtype=torch.uint8, device=x.device)
        lib.adr_maxpool(dcode(x.dtype), ctypes.c_void_p(vx[1]), vx[2], ctypes.c_void_p(yp), ycs, fptr(arg),
                        N, H, W, C, k, stream())
        ctx.save_for_backward(arg)
        ctx.meta = (k, x.shape, x.dtype)
        ctx.sink = _sink_of(x)
        return y if box is None else y[:, :]

    @staticmethod
    def backward(ctx, dy):
        (arg,) = ctx.saved_tensors
        k, shape, dtype = ctx.meta
        N, C, H, W = shape
        vd = _v(dy)
        dx, acc = _dx_dst(ctx, (N, C, H, W), dtype, dy.device)
        lib.adr_maxpool_bwd(dcode(dtype), ctypes.c_void_p(vd[1]), vd[2], fptr(arg), ctypes.c_void_p(dx.data_ptr()),
                            dx.stride(3), N, H, W, C, k, acc, stream())
        return (None if ctx.sink is not None else dx), None, None


def maxpool(x, k, out=None):
    return MaxPoolFn.apply(x, k, None if out is None else OutBox(out))


class MLCAFn(torch.autograd.Function):
    """res + MLCA(y) (block.py:1540-1594) — 3 fused kernels forward, 3 (+2 tiny) backward."""

    @staticmethod
    def forward(ctx, y, res, wl, wg, local_weight, box=None):
        vy = _v(y)
        N, C, H, W = y.shape
        dev = y.device
        f = lambda *s: torch.empty(s, dtype=torch.float32, device=dev)  # noqa: E731
        local, att, sig_l, sig_g = f(N, 25, C), f(N, 25, C), f(N, 25 * C), f(N, C)
        out, op, ocs = _out_view(box, N, C, H, W, y.dtype, dev)  # a concat slot when the caller passes one
        vr = _v(res) if res is not None else None
        wlf, wgf = wl.detach().float().contiguous().view(-1), wg.detach().float().contiguous().view(-1)
        k = wlf.numel()
        lib.adr_mlca_fwd(dcode(y.dtype), ctypes.c_void_p(vy[1]), vy[2], ctypes.c_void_p(vr[1]) if vr else None,
                         vr[2] if vr else 0, ctypes.c_void_p(op), ocs, N, H, W, C, fptr(wlf), fptr(wgf), k,
                         float(local_weight), fptr(local), fptr(att), fptr(sig_l), fptr(sig_g), stream())
        ctx.save_for_backward(vy[0], wlf, wgf, local, att, sig_l, sig_g)
        ctx.meta = (local_weight, res is not None, wl.shape, wg.shape)
        ctx.pwl, ctx.pwg = wl, wg
        ctx.sres = getattr(res, "_adr_sink", None) if res is not None else None
        return out if box is None else out[:, :]

    @staticmethod
    def backward(ctx, dout):
        y, wlf, wgf, local, att, sig_l, sig_g = ctx.saved_tensors
        lw, has_res, wls, wgs = ctx.meta
        N, C, H, W = y.shape
        vd, vy = _v(dout), _v(y)
        dy = _new_like(y)
        k = wlf.numel()
        wsb = lib.adr_mlca_bwd_workspace(N, C, k)
        ws = torch.empty(wsb // 4 + 1, dtype=torch.float32, device=y.device)
        tl, tg = _target(ctx.pwl), _target(ctx.pwg)
        # both Conv1d weight gradients land in the arena: leave the per-image rows and reduce them at the deferred
        # flush with the other partial sums (no sum launch, no temporaries, no axpy entries)
        defer = (_DEFER_MLCA and _dfr() is not None and _TIMING is None and tl is not None and tg is not None
                 and tl is not tg)
        dwl = dwg = None
        if not defer:
            dwl = torch.empty(k, dtype=torch.float32, device=y.device)
            dwg = torch.empty(k, dtype=torch.float32, device=y.device)
        lib.adr_mlca_bwd(dcode(y.dtype), ctypes.c_void_p(vy[1]), vy[2], ctypes.c_void_p(vd[1]), vd[2],
                         ctypes.c_void_p(dy.data_ptr()), C, N, H, W, C, fptr(wlf), fptr(wgf), k, float(lw),
                         fptr(local), fptr(att), fptr(sig_l), fptr(sig_g), fptr(dwl), fptr(dwg), fptr(ws), wsb,
                         stream())
        dres = _defer_pass(ctx.sres, dout) if has_res else None
        if defer:
            rows = ws[2 * N * 25 * C:2 * N * 25 * C + 2 * N * k]
            for which, t in ((0, tl), (1, tg)):
                _dfr().add_psum(rows, N, k, which, fptr(_grad_buf(t)), 1)
                t._adr_used = True
            return dy, dres, None, None, None, None
        return dy, dres, sink(ctx.pwl, dwl.view(wls)), sink(ctx.pwg, dwg.view(wgs)), None, None


def mlca(y, res, wl, wg, local_weight=0.5, out=None):
    return MLCAFn.apply(y, res, wl, wg, local_weight, None if out is None else OutBox(out))


class AxisMeanFn(torch.autograd.Function):
    """Row means over W and column means over H, written as NHWC 'images':
    layout 'ela'   -> (2N, C, L, 1): rows [0,N) hold the H-means (L=H), rows [N,2N) the W-means (needs H == W)
    layout 'coord' -> (N, C, H+W, 1): per image rows [0,H) H-means then [H,H+W) W-means (CoordAtt cat)."""

    @staticmethod
    def forward(ctx, x, layout):
        vx = _v(x)
        N, C, H, W = x.shape
        dev = x.device
        if layout == "ela":
            if H != W:
                raise RuntimeError("ELA_HSFPN shares one Conv1d over both axes; this build needs H == W")
            out = empty_act(2 * N, C, H, 1, x.dtype, dev)
            oh, ohn = out.data_ptr(), H * C
            ow, own = out.data_ptr() + N * H * C * out.element_size(), W * C
        else:
            out = empty_act(N, C, H + W, 1, x.dtype, dev)
            oh, ohn = out.data_ptr(), (H + W) * C
            ow, own = out.data_ptr() + H * C * out.element_size(), (H + W) * C
        lib.adr_axis_mean(dcode(x.dtype), ctypes.c_void_p(vx[1]), vx[2], N, H, W, C, ctypes.c_void_p(oh), ohn,
                          ctypes.c_void_p(ow), own, stream())
        ctx.meta = (layout, x.shape, x.dtype)
        ctx.sink = _sink_of(x)
        return out

    @staticmethod
    def backward(ctx, dy):
        layout, shape, dtype = ctx.meta
        N, C, H, W = shape
        dy = dy.contiguous(memory_format=torch.channels_last) if not _is_dense_nhwc(dy) else dy
        es = dy.element_size()
        if layout == "ela":
            dh, dhn, dw, dwn = dy.data_ptr(), H * C, dy.data_ptr() + N * H * C * es, W * C
        else:
            dh, dhn, dw, dwn = dy.data_ptr(), (H + W) * C, dy.data_ptr() + H * C * es, (H + W) * C
        dx, acc = _dx_dst(ctx, (N, C, H, W), dtype, dy.device)
        lib.adr_axis_mean_bwd(dcode(dtype), ctypes.c_void_p(dh), dhn, ctypes.c_void_p(dw), dwn,
                              ctypes.c_void_p(dx.data_ptr()), dx.stride(3), N, H, W, C, acc, stream())
        return (None if ctx.sink is not None else dx), None


def _is_dense_nhwc(t):
    n, c, h, w = t.shape
    return t.stride() == (h * w * c, 1, w * c, c) or t.is_contiguous(memory_format=torch.channels_last)


def axis_mean(x, layout):
    return AxisMeanFn.apply(x, layout)


class GateFn(torch.autograd.Function):
    """out = (x if x is not None else 1) * a_h[n,h,c] * a_w[n,w,c], with a = the (.., L, 1) planes produced in
    the AxisMeanFn layouts ('ela': a is (2N, C, L, 1); 'coord': a_h / a_w are (N, C, H+W, 1) tensors)."""

    @staticmethod
    def forward(ctx, x, ah_t, aw_t, layout, shape):
        N, C, H, W = shape
        dtype = ah_t.dtype
        ah_t = ah_t if _is_dense_nhwc(ah_t) else ah_t.contiguous(memory_format=torch.channels_last)
        aw_t = aw_t if _is_dense_nhwc(aw_t) else aw_t.contiguous(memory_format=torch.channels_last)
        es = ah_t.element_size()
        if layout == "ela":
            ah, ahn = ah_t.data_ptr(), H * C
            aw, awn = aw_t.data_ptr() + N * H * C * es, W * C
        else:
            ah, ahn = ah_t.data_ptr(), (H + W) * C
            aw, awn = aw_t.data_ptr() + H * C * es, (H + W) * C
        vx = _v(x) if x is not None else (None, 0, 0)
        out = empty_act(N, C, H, W, dtype, ah_t.device)
        lib.adr_gate(dcode(dtype), ctypes.c_void_p(vx[1]) if x is not None else None, vx[2], ctypes.c_void_p(ah), ahn,
                     ctypes.c_void_p(aw), awn, ctypes.c_void_p(out.data_ptr()), C, N, H, W, C, stream())
        ctx.save_for_backward(*( [vx[0]] if x is not None else []), ah_t, aw_t)
        ctx.meta = (layout, shape, x is not None, (ah, ahn, aw, awn))
        ctx.sink = _sink_of(x) if x is not None else None
        return out

    @staticmethod
    def backward(ctx, dout):
        layout, shape, has_x, (ah, ahn, aw, awn) = ctx.meta
        saved = ctx.saved_tensors
        x = saved[0] if has_x else None
        ah_t, aw_t = saved[-2], saved[-1]
        N, C, H, W = shape
        vd = _v(dout)
        dtype = ah_t.dtype
        es = ah_t.element_size()
        if layout == "ela":
            da = torch.empty_like(ah_t, memory_format=torch.channels_last)
            dah, dahn, daw, dawn = da.data_ptr(), H * C, da.data_ptr() + N * H * C * es, W * C
            dah_t = daw_t = None
        else:
            # the kernel zeroes the rows the gate does not use (dah rows H.., daw rows ..H): no fill launches
            dah_t = torch.empty_like(ah_t, memory_format=torch.channels_last)
            daw_t = torch.empty_like(aw_t, memory_format=torch.channels_last)
            dah, dahn = dah_t.data_ptr(), (H + W) * C
            daw, dawn = daw_t.data_ptr() + H * C * es, (H + W) * C
        dx, acc = _dx_dst(ctx, (N, C, H, W), dtype, dout.device) if has_x else (None, 0)
        vx = _v(x) if has_x else (None, 0, 0)
        _gate_bwd(dcode(dtype), vx[1] if has_x else None, vx[2], ah, ahn, aw, awn, vd[1], vd[2],
                  dx.data_ptr() if has_x else None, dx.stride(3) if has_x else C, dah, dahn, daw, dawn, N, H, W, C,
                  acc, int(layout != "ela"), dout.device)
        if ctx.sink is not None:
            dx = None
        if layout == "ela":
            return dx, da, None, None, None
        return dx, dah_t, daw_t, None, None


def _gate_bwd(dt, xp, xcs, ah, ahn, aw, awn, dp, dcs, dx, dxcs, dah, dahn, daw, dawn, N, H, W, C, acc, zero_other,
              dev):
    """dx (+)= dout * a_h * a_w and the a_h / a_w gradients (adr_gate_bwd: per-row / per-column reductions, then dx;
    a one-pass variant with band-partial column sums measured slower: 0.40 vs 0.31 ms per step)."""
    lib.adr_gate_bwd(dt, ctypes.c_void_p(xp) if xp is not None else None, xcs, ctypes.c_void_p(ah), ahn,
                     ctypes.c_void_p(aw), awn, ctypes.c_void_p(dp), dcs,
                     ctypes.c_void_p(dx) if dx is not None else None, dxcs, ctypes.c_void_p(dah), dahn,
                     ctypes.c_void_p(daw), dawn, N, H, W, C, acc, zero_other, stream())


def gate(x, ah, aw, layout, shape):
    return GateFn.apply(x, ah, aw, layout, shape)


# ---------------------------------------------------------------------------------------------------------
# head helpers
# ---------------------------------------------------------------------------------------------------------


class GapFn(torch.autograd.Function):
    """Global average pool -> (N, C) fp32 (F.adaptive_avg_pool2d(x, 1), head.py:1142)."""

    @staticmethod
    def forward(ctx, x):
        N, C, H, W = x.shape
        s = _reduce_dot(None, x, False, False, which=1).view(N, C)
        ctx.meta = (x.shape, x.dtype)
        return _vec_affine(s, 1.0 / (H * W))

    @staticmethod
    def backward(ctx, dg):
        (N, C, H, W), dtype = ctx.meta
        dx = empty_act(N, C, H, W, dtype, dg.device)
        dgc = dg.float().contiguous()
        lib.adr_bcast_fill(dcode(dtype), fptr(dgc), C, 1, 1.0 / (H * W), ctypes.c_void_p(dx.data_ptr()), C, N, H * W,
                           C, 0, stream())
        return dx


def _vec_affine(v, s):
    """out = v * s for a small contiguous fp32 vector (adr_bcast_fill on a one-pixel 'image')."""
    n = v.numel()
    out = torch.empty_like(v)
    lib.adr_bcast_fill(F32, fptr(v.contiguous()), 0, 1, float(s), fptr(out), n, 1, 1, n, 0, stream())
    return out


def gap(x):
    return GapFn.apply(x)


class GateMLPFn(torch.autograd.Function):
    """act2(W2 act1(W1 v + b1) + b2) per image on pooled vectors v (N, Cin) fp32."""

    ACTS = {"none": 0, "relu": 3, "sigmoid": 4, "softmax": 6}

    @staticmethod
    def forward(ctx, v, W1, b1, W2, b2, act1, act2):
        N, Cin = v.shape
        H1, H2 = W1.shape[0], W2.shape[0]
        vv = v.float().contiguous()
        w1 = W1.detach().float().contiguous().view(H1, -1)
        w2 = W2.detach().float().contiguous().view(H2, -1)
        b1f = b1.detach().float().contiguous() if b1 is not None else None
        b2f = b2.detach().float().contiguous() if b2 is not None else None
        hidden = torch.empty(N, H1, dtype=torch.float32, device=v.device)
        out = torch.empty(N, H2, dtype=torch.float32, device=v.device)
        a1, a2 = GateMLPFn.ACTS[act1], GateMLPFn.ACTS[act2]
        lib.adr_gate_mlp(fptr(vv), 1.0, N, Cin, fptr(w1), fptr(b1f), H1, a1, fptr(w2), fptr(b2f), H2, a2,
                         fptr(hidden), fptr(out), stream())
        ctx.save_for_backward(vv, w1, w2, hidden, out)
        ctx.meta = (a1, a2, W1.shape, W2.shape, b1 is not None, b2 is not None)
        ctx.params = (W1, b1, W2, b2)
        return out

    @staticmethod
    def backward(ctx, dout):
        vv, w1, w2, hidden, out = ctx.saved_tensors
        a1, a2, s1, s2, hb1, hb2 = ctx.meta
        N, Cin = vv.shape
        H1, H2 = w1.shape[0], w2.shape[0]
        d = dout.float().contiguous()
        dev = vv.device
        din = torch.empty_like(vv)
        W1p, b1p, W2p, b2p = ctx.params
        dW1, p1, acc = grad_dst(W1p, H1 * Cin, dev)
        dW2, p2, acc2 = grad_dst(W2p, H2 * H1, dev)
        db1, pb1, acc3 = grad_dst(b1p, H1, dev) if hb1 else (None, None, acc)
        db2, pb2, acc4 = grad_dst(b2p, H2, dev) if hb2 else (None, None, acc)
        if len({acc, acc2, acc3, acc4}) != 1:
            raise RuntimeError("gate_mlp: parameter gradients must share one destination kind")
        lib.adr_gate_mlp_bwd(fptr(vv), 1.0, N, Cin, fptr(w1), H1, a1, fptr(w2), H2, a2, fptr(hidden), fptr(out),
                             fptr(d), fptr(din), p1, pb1, p2, pb2, acc, stream())
        return (din, grad_ret(W1p, dW1), grad_ret(b1p, db1) if hb1 else None, grad_ret(W2p, dW2),
                grad_ret(b2p, db2) if hb2 else None, None, None)


def gate_mlp(v, W1, b1, W2, b2, act1, act2):
    return GateMLPFn.apply(v, W1, b1, W2, b2, act1, act2)


def padded_conv2d(x, w, b, stride, pad, kpad):
    """Dense conv whose output channels are zero-padded to `kpad` (27 -> 32 offset/mask conv; 1 -> 8 cls_prob)
    so every NHWC row stays 16-byte aligned; returns the (N, kpad, H, W) tensor (extra channels are 0)."""
    return PaddedConvFn.apply(x, w, b, stride, pad, kpad)


_PBIAS = {}


def _padded_bias(b, K, kpad, dev):
    """fp32 bias zero-padded to kpad channels: a persistent buffer per (bias, kpad) whose padding stays zero; each
    call copies the current K values in (one launch; the optimizer updates the bias in place between steps)."""
    key = (None if b is None else id(b), kpad, dev)
    hit = _PBIAS.get(key)
    if hit is None or (b is not None and hit[0] is not b):
        hit = _PBIAS[key] = (b, torch.zeros(kpad, dtype=torch.float32, device=dev))
    if b is not None:
        lib.adr_cast(F32, fptr(b.detach().float().contiguous()), F32, fptr(hit[1]), K, stream())
    return hit[1]


class PaddedConvFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, b, stride, pad, kpad):
        dtype = x.dtype
        x, xp, xcs = nhwc(x)
        N, C, H, W = x.shape
        K, _, R, S = w.shape
        RS = R * S
        if dtype == torch.bfloat16:
            wp, wt = pack_weight2(w, dtype, kpad=kpad)
        else:
            wp, wt = torch.empty(kpad * RS * C, dtype=dtype, device=x.device), None
            zero_(wp)
            wf = w.detach().float().contiguous()
            lib.adr_pack_weight(dcode(dtype), fptr(wf), fptr(wp), K, C, C, RS, 0, stream())
        bp = _padded_bias(b, K, kpad, x.device)
        d, Ho, Wo = conv_desc(N, H, W, C, xcs, kpad, R, S, stride, stride, pad, pad, kpad, dtype)
        y = empty_act(N, kpad, Ho, Wo, dtype, x.device)
        conv_fwd(d, xp, wp.data_ptr(), fptr(bp), y.data_ptr())
        ctx.save_for_backward(x, wp, wt)
        ctx.meta = (stride, pad, kpad, w.shape, b is not None)
        ctx.pw, ctx.pb = w, b
        return y

    @staticmethod
    def backward(ctx, dy):
        x, wp, wt = ctx.saved_tensors
        stride, pad, kpad, wshape, has_b = ctx.meta
        dy, dyp, dycs = nhwc(dy.to(x.dtype) if dy.dtype != x.dtype else dy)
        N, C, H, W = x.shape
        K, _, R, S = wshape
        x, xp, xcs = nhwc(x)
        dx = dw = db = None
        if ctx.needs_input_grad[0]:
            dx = empty_act(N, C, H, W, x.dtype, x.device)
            d2, _, _ = conv_desc(N, H, W, C, C, kpad, R, S, stride, stride, pad, pad, dycs, x.dtype)
            conv_dgrad(d2, dyp, (wp, wt), None, dx.data_ptr())
        d, Ho, Wo = conv_desc(N, H, W, C, xcs, kpad, R, S, stride, stride, pad, pad, dycs, x.dtype)
        if ctx.needs_input_grad[1]:
            dw = wgrad_param(ctx.pw, d, xp, dyp, kpad, C, R * S, wshape, 0, x.device)  # first K rows of [kpad][RS][C]
        if has_b and ctx.needs_input_grad[2]:
            db = sink(ctx.pb, _bias_grad(dy, kpad, N, Ho * Wo, dycs)[:K])
        return dx, dw, db, None, None, None


def _dcn_fused(dtype, C, Cout, omcs):
    """The bf16 fused DCN kernels (adr_dcn.hip) cover the head's shapes; fp32 parity mode and other shapes take
    im2col + GEMM + the deterministic col2im."""
    return _DCN_FUSED and dtype == torch.bfloat16 and C % 64 == 0 and Cout % 64 == 0 and Cout <= 256 and \
        omcs % 8 == 0 and omcs >= 32


_DCN_FUSED = bool(int(__import__("os").environ.get("ADR_DCN_FUSED", "1")))  # 0: im2col path (A/B only)


_DCN_FAR = {}  # device -> (fp32 far-corner buffer, tile flags), grown to the largest shape seen
_DCN_FAR_RETIRED = []  # outgrown buffers: a captured graph may still address them


# 1: a freshly zeroed far-corner pair per backward call (its memset also leaves the buffer in the Infinity Cache
# right before the kernel's far-corner atomics); 0: one persistent pair per device (the kernels leave it zero)
_DCN_FAR_FRESH = bool(int(__import__("os").environ.get("ADR_DCN_FAR_FRESH", "0")))


def _dcn_far_scratch(dev, N, H, W, C):
    """Persistent zeroed scratch of adr_dcn_bwd_bf16: the fp32 far-corner buffer and the tile flags. The kernels
    leave both zero again, so ONE pair per device serves every level, shape, step and graph replay (calls are
    stream-ordered); a call uses a prefix view of it."""
    if _DCN_FAR_FRESH:
        return (torch.zeros(N * H * W * C, dtype=torch.float32, device=dev),
                torch.zeros(int(lib.adr_dcn_bwd_tiles(N, H, W)), dtype=torch.int32, device=dev))
    key = str(dev)
    n, nt = N * H * W * C, int(lib.adr_dcn_bwd_tiles(N, H, W))
    cur = _DCN_FAR.get(key)
    if cur is None or cur[0].numel() < n or cur[1].numel() < nt:
        if cur is not None:
            _DCN_FAR_RETIRED.append(cur)
            n, nt = max(n, cur[0].numel()), max(nt, cur[1].numel())
        cur = (torch.zeros(n, dtype=torch.float32, device=dev), torch.zeros(nt, dtype=torch.int32, device=dev))
        _DCN_FAR[key] = cur
    return cur[0][:N * H * W * C], cur[1][:int(lib.adr_dcn_bwd_tiles(N, H, W))]


def _dcn_far_scratch_levels(dev, N, dims, C):
    """Per-level disjoint views of the persistent far-corner scratch, for the levels-in-one-launch backward."""
    n = sum(N * H * W * C for H, W in dims)
    nt = sum(int(lib.adr_dcn_bwd_tiles(N, H, W)) for H, W in dims)
    key = str(dev)
    cur = _DCN_FAR.get(key)
    if _DCN_FAR_FRESH:
        cur = (torch.zeros(n, dtype=torch.float32, device=dev), torch.zeros(nt, dtype=torch.int32, device=dev))
    # compare against the FULL persistent pair (not a prefix view), so it grows only when really too small
    elif cur is None or cur[0].numel() < n or cur[1].numel() < nt:
        if cur is not None:
            _DCN_FAR_RETIRED.append(cur)
            n, nt = max(n, cur[0].numel()), max(nt, cur[1].numel())
        _DCN_FAR[key] = cur = (torch.zeros(n, dtype=torch.float32, device=dev),
                               torch.zeros(nt, dtype=torch.int32, device=dev))
    f, g = cur
    out, o, ot = [], 0, 0
    for H, W in dims:
        k, kt = N * H * W * C, int(lib.adr_dcn_bwd_tiles(N, H, W))
        out.append((f[o:o + k], g[ot:ot + kt]))
        o, ot = o + k, ot + kt
    return out


class DcnLevelStruct(ctypes.Structure):
    """adr_dcn_level (include/adr.h)."""
    _fields_ = [(n, ctypes.c_void_p) for n in ("x", "om", "dy", "y", "dx", "dom", "dxf", "flags", "part")] + [
        (n, ctypes.c_int) for n in ("H", "W", "splits", "pad_")]


# the AYHead's DCN levels in one launch per direction (adr_dcn_*_bf16_levels; ADR_DCN_LEVELS=0: one per level)
DCN_LEVELS = bool(int(__import__("os").environ.get("ADR_DCN_LEVELS", "1")))


def _dcn_work(N, H, W, C, Cout, es=2):
    """Algorithmic (bytes, flops) of one DCN pass: x, the 27 offset/mask channels, the weight and y (or dy) once."""
    pix = N * H * W
    return es * (pix * (C + 27 + Cout) + 9 * C * Cout), 2 * pix * 9 * C * Cout


class DCNFn(torch.autograd.Function):
    """mmcv ModulatedDeformConv2d(C, Cout, 3, 1, 1, bias=False) with offsets / mask logits from `om`
    (head.py:751-782). bf16: fused sampling + MFMA kernels, no column matrix in HBM (adr_dcn.hip). fp32 parity
    mode: im2col -> GEMM, and a deterministic col2im (bitwise repeatable)."""

    @staticmethod
    def forward(ctx, x, om, w):
        dtype = x.dtype
        x, xp, xcs = nhwc(x)
        om, omp, omcs = nhwc(om)
        N, C, H, W = x.shape
        Cout = w.shape[0]
        y = empty_act(N, Cout, H, W, dtype, x.device)
        ctx.fused = _dcn_fused(dtype, C, Cout, omcs)
        ctx.fused_bwd = ctx.fused and C == Cout and C in (64, 128, 256)
        if ctx.fused:
            wp = pack_weight2(w, dtype)[0]  # KRSC [co][tap][c]
            tok = _t0("adr::dcn_fwd_kernel(adr::DcnArgs)", *_dcn_work(N, H, W, C, Cout),
                      f"dcn fwd n{N} {H}x{W} c{C}->{Cout}" if _TIMING is not None else "", _reps())
            for _ in range(_reps()):
                lib.adr_dcn_fwd_bf16(ctypes.c_void_p(xp), xcs, ctypes.c_void_p(omp), omcs, fptr(wp),
                                     ctypes.c_void_p(y.data_ptr()), Cout, N, H, W, C, Cout, stream())
            _t1(tok)
            ctx.save_for_backward(x, om, w)
        else:
            cols = torch.empty(N * H * W * 9 * C, dtype=dtype, device=x.device)
            lib.adr_dcn_im2col(dcode(dtype), ctypes.c_void_p(xp), xcs, ctypes.c_void_p(omp), omcs, fptr(cols), N, H, W,
                               C, stream())
            wp = pack_weight(w, dtype)  # KRSC [co][tap][c] == 1x1 weight over the [tap][c] columns
            d, _, _ = conv_desc(N, H, W, 9 * C, 9 * C, Cout, 1, 1, 1, 1, 0, 0, Cout, dtype)
            conv_fwd(d, cols.data_ptr(), wp.data_ptr(), None, y.data_ptr())
            ctx.save_for_backward(x, om, cols, w)
        ctx.pw = w
        return y

    @staticmethod
    def backward(ctx, dy):
        cols = None
        if ctx.fused:
            x, om, w = ctx.saved_tensors
        else:
            x, om, cols, w = ctx.saved_tensors
        dtype = x.dtype
        _, xp, xcs = nhwc(x)
        _, omp, omcs = nhwc(om)
        dy, dyp, dycs = nhwc(dy.to(dtype) if dy.dtype != dtype else dy)
        N, C, H, W = x.shape
        Cout = w.shape[0]
        dev = x.device
        wt = torch.empty(9 * C * Cout, dtype=dtype, device=dev)  # W^T [(tap*C + c)][co]
        lib.adr_dcn_weight_t(dcode(dtype), fptr(w.detach().float().contiguous()), fptr(wt), Cout, C, stream())
        dw = None
        if ctx.fused and not ctx.fused_bwd:  # fused forward, other shapes: rebuild the columns for the GEMMs
            cols = torch.empty(N * H * W * 9 * C, dtype=dtype, device=dev)
            lib.adr_dcn_im2col(dcode(dtype), ctypes.c_void_p(xp), xcs, ctypes.c_void_p(omp), omcs, fptr(cols), N, H,
                               W, C, stream())
        if ctx.fused_bwd:
            # gathered by destination tile: bf16 dx written once, dom rows written whole (adr_dcn.hip)
            dx = empty_act(N, C, H, W, dtype, dev)
            dom = empty_act(N, om.shape[1], H, W, dtype, dev)
            dxf, flags = _dcn_far_scratch(dev, N, H, W, C)
            nb, fl = _dcn_work(N, H, W, C, Cout)
            tok = _t0("adr::dcn_bwd_kernel(adr::DcnArgs)", nb + 2 * N * H * W * C, 2 * fl,
                      f"dcn bwd n{N} {H}x{W} c{C}->{Cout}" if _TIMING is not None else "")
            lib.adr_dcn_bwd_bf16(ctypes.c_void_p(xp), xcs, ctypes.c_void_p(omp), omcs, ctypes.c_void_p(dyp), dycs,
                                 fptr(wt), ctypes.c_void_p(dx.data_ptr()), C, ctypes.c_void_p(dom.data_ptr()),
                                 om.shape[1], fptr(dxf), fptr(flags), N, H, W, C, Cout, stream())
            _t1(tok)
            if ctx.needs_input_grad[2]:
                splits = lib.adr_dcn_wgrad_bf16_splits(N, H, W, C, Cout)
                stride = Cout * 9 * C
                ws = torch.empty(splits * stride, dtype=torch.float32, device=dev)
                rep = _reps()
                tok = _t0("adr::dcn_wgrad_kernel(adr::DcnArgs)", nb + 4 * splits * stride, fl,
                          f"dcn wgrad/{splits} n{N} {H}x{W} c{C}->{Cout}" if _TIMING is not None else "", rep)
                for _ in range(rep):
                    lib.adr_dcn_wgrad_bf16(ctypes.c_void_p(xp), xcs, ctypes.c_void_p(omp), omcs,
                                           ctypes.c_void_p(dyp), dycs, fptr(ws), splits, N, H, W, C, Cout,
                                           stream())
                _t1(tok)
                out, ptr, acc = grad_dst(ctx.pw, stride, dev)
                if _dfr() is not None and acc and _TIMING is None:
                    _dfr().add(ws, stride, splits, ptr, Cout, C, C, 9, 0, acc)
                else:
                    lib.adr_wgrad_reduce_unpack(fptr(ws), stride, splits, ptr, Cout, C, C, 9, 0, acc, stream())
                dw = grad_ret(ctx.pw, out)
        else:
            dx32 = zero_(torch.empty(N * H * W * C, dtype=torch.float32, device=dev))
            dom = zero_(empty_act(N, om.shape[1], H, W, dtype, dev))
            # dcols = dy x W^T  (1x1 GEMM: Cin = Cout, K = 9C)
            dcols = torch.empty(N * H * W * 9 * C, dtype=dtype, device=dev)
            d, _, _ = conv_desc(N, H, W, Cout, dycs, 9 * C, 1, 1, 1, 1, 0, 0, 9 * C, dtype)
            conv_fwd(d, dyp, wt.data_ptr(), None, dcols.data_ptr())
            if ctx.needs_input_grad[2]:
                dwd, _, _ = conv_desc(N, H, W, 9 * C, 9 * C, Cout, 1, 1, 1, 1, 0, 0, dycs, dtype)
                dw = wgrad_param(ctx.pw, dwd, cols.data_ptr(), dyp, Cout, 9 * C, 1, w.shape, 0, dev, keep=(cols, dy))
            lib.adr_dcn_col2im(dcode(dtype), ctypes.c_void_p(xp), xcs, ctypes.c_void_p(omp), omcs, fptr(dcols),
                               fptr(dx32), ctypes.c_void_p(dom.data_ptr()), om.shape[1], N, H, W, C,
                               int(dtype == torch.float32), stream())
            dx = empty_act(N, C, H, W, dtype, dev)
            lib.adr_cast(F32, fptr(dx32), dcode(dtype), ctypes.c_void_p(dx.data_ptr()), N * H * W * C, stream())
        return dx, dom, dw


def dcn(x, om, w):
    return DCNFn.apply(x, om, w)


class MulPixelFn(torch.autograd.Function):
    """x * p[:, 0:1] (per-pixel scalar from channel 0 of p)."""

    @staticmethod
    def forward(ctx, x, p):
        vx, vp = _v(x), _v(p)
        N, C, H, W = x.shape
        out = _new_like(vx[0])
        lib.adr_mul_pixel(dcode(x.dtype), ctypes.c_void_p(vx[1]), vx[2], ctypes.c_void_p(vp[1]), vp[2],
                          ctypes.c_void_p(out.data_ptr()), C, N * H * W, C, stream())
        ctx.save_for_backward(vx[0], vp[0])
        return out

    @staticmethod
    def backward(ctx, dout):
        x, p = ctx.saved_tensors
        vx, vp, vd = _v(x), _v(p), _v(dout)
        N, C, H, W = x.shape
        dx = _new_like(x)
        dp = _new_like(p)  # adr_mul_pixel_bwd writes the whole row (channel 0, zeros after it)
        lib.adr_mul_pixel_bwd(dcode(x.dtype), ctypes.c_void_p(vx[1]), vx[2], ctypes.c_void_p(vp[1]), vp[2],
                              ctypes.c_void_p(vd[1]), vd[2], ctypes.c_void_p(dx.data_ptr()), C,
                              ctypes.c_void_p(dp.data_ptr()), p.shape[1], N * H * W, C, stream())
        return dx, dp


def mul_pixel(x, p):
    return MulPixelFn.apply(x, p)


def detect_decode(feats, strides, nc, reg_max=16):
    """Eval-branch decode of AYHead (head.py:1181-1204) -> y (B, 4+nc, A) fp32."""
    vs = [_v(f) for f in feats]
    B = feats[0].shape[0]
    A = sum(f.shape[2] * f.shape[3] for f in feats)
    y = torch.empty(B, 4 + nc, A, dtype=torch.float32, device=feats[0].device)
    (f0, f1, f2) = vs
    lib.adr_detect_decode(dcode(feats[0].dtype), ctypes.c_void_p(f0[1]), ctypes.c_void_p(f1[1]), ctypes.c_void_p(f2[1]),
                          f0[2], f1[2], f2[2], feats[0].shape[2], feats[0].shape[3], feats[1].shape[2],
                          feats[1].shape[3], feats[2].shape[2], feats[2].shape[3], float(strides[0]), float(strides[1]),
                          float(strides[2]), B, nc, reg_max, fptr(y), stream())
    return y


# ---------------------------------------------------------------------------------------------------------
# C2PTSSA helpers
# ---------------------------------------------------------------------------------------------------------


class DWConvFn(torch.autograd.Function):
    """Depthwise k x k conv (groups = C), stride 1, pad k//2, optional bias."""

    @staticmethod
    def forward(ctx, x, w, b, k):
        vx = _v(x)
        N, C, H, W = x.shape
        wf = w.detach().float().contiguous()
        bf = b.detach().float().contiguous() if b is not None else None
        y = _new_like(vx[0])
        lib.adr_dwconv_fwd(dcode(x.dtype), ctypes.c_void_p(vx[1]), vx[2], fptr(wf), fptr(bf),
                           ctypes.c_void_p(y.data_ptr()), C, N, H, W, C, k, stream())
        ctx.save_for_backward(vx[0], wf)
        ctx.meta = (k, w.shape, b is not None)
        ctx.pw, ctx.pb = w, b
        ctx.sink = _sink_of(x)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, wf = ctx.saved_tensors
        k, wshape, has_b = ctx.meta
        N, C, H, W = x.shape
        vx, vd = _v(x), _v(dy)
        dx, acc = _dx_dst(ctx, (N, C, H, W), x.dtype, x.device) if ctx.needs_input_grad[0] else (None, 0)
        dw, pdw, dacc = grad_dst(ctx.pw, C * k * k, x.device) if ctx.needs_input_grad[1] else (None, None, 0)
        wsb = lib.adr_dwconv_wgrad_workspace(N, H, W, C, k)
        ws = torch.empty(wsb // 4 + 1, dtype=torch.float32, device=x.device)
        # weight gradient into the arena: the partial rows now, their reduction batched at the deferred flush
        # (adr_wgrad_reduce_batched with K = 1, RS = k*k: the [C][k*k] parameter layout)
        defer = pdw is not None and dacc and _dfr() is not None and _TIMING is None and wsb <= DEFER_MAX_BYTES
        lib.adr_dwconv_bwd(dcode(x.dtype), ctypes.c_void_p(vx[1]), vx[2], ctypes.c_void_p(vd[1]), vd[2], fptr(wf),
                           ctypes.c_void_p(dx.data_ptr()) if dx is not None else None,
                           dx.stride(3) if dx is not None else C, None if defer else pdw, N, H, W, C, k, acc, dacc,
                           fptr(ws), wsb, stream())
        db, fused = None, False
        if defer:
            chunks = ctypes.c_int(0)
            if (has_b and ctx.needs_input_grad[2] and _fuse_wg_bias() and
                    lib.adr_dwconv_wgrad_bias_fusable(dcode(x.dtype), H, W, C, k, vx[2], vd[2])):
                # the bias gradient's column sums from the staged dy slab of the same launch
                bpart = torch.empty(N * 2 * C, dtype=torch.float32, device=x.device)
                lib.adr_dwconv_wgrad_partials_bias(dcode(x.dtype), ctypes.c_void_p(vx[1]), vx[2],
                                                   ctypes.c_void_p(vd[1]), vd[2], N, H, W, C, k, fptr(ws), wsb,
                                                   fptr(bpart), ctypes.byref(chunks), stream())
                db, fused = _bias_rows(ctx.pb, C, N, bpart, x.device), True
            else:
                lib.adr_dwconv_wgrad_partials(dcode(x.dtype), ctypes.c_void_p(vx[1]), vx[2], ctypes.c_void_p(vd[1]),
                                              vd[2], N, H, W, C, k, fptr(ws), wsb, ctypes.byref(chunks), stream())
            _dfr().add(ws, k * k * C, chunks.value, pdw, 1, C, C, k * k, 0, dacc)
        if has_b and ctx.needs_input_grad[2] and not fused:
            db = _bias_grad(vd[0], C, N, H * W, vd[2], ctx.pb)
        return (None if ctx.sink is not None else dx), grad_ret(ctx.pw, dw), db, None


def dwconv(x, w, b, k):
    return DWConvFn.apply(x, w, b, k)


def dwconv_bn_act_eval(x, w, k, bn, act: str, out=None):
    """Inference DWConv-BN-act (no autograd) in one launch (adr_dwconv_fwd_act): the BatchNorm scale folded into
    the staged fp32 taps, the shift as the bias, the activation before the store — Conv.forward_fuse after
    fuse_conv_and_bn on a depthwise Conv (nn/modules/conv.py:52-54, 101-106). None when not applicable."""
    if x.dtype != torch.bfloat16 or torch.is_grad_enabled():
        return None
    N, C, H, W = x.shape
    if not lib.adr_dwconv_fwd_act_supported(H, W, C, k):
        return None
    vx = _v(x)
    y, yp, ycs = _out_view(None if out is None else OutBox(out), N, C, H, W, x.dtype, x.device)
    wf = w.detach().float().contiguous()
    scale, shift = _bn_eval_coefs(bn, x.device)
    lib.adr_dwconv_fwd_act(ctypes.c_void_p(vx[1]), vx[2], fptr(wf), fptr(scale), fptr(shift), ACT[act],
                           ctypes.c_void_p(yp), ycs, N, H, W, C, k, stream())
    return y if out is None else out


class ADyTFn(torch.autograd.Function):
    """AdaptiveDynamicTanh apply (block.py:2547-2575) given the softmax importance imp (N, 3)."""

    @staticmethod
    def forward(ctx, x, alphas, imp, w, b):
        vx = _v(x)
        N, C, H, W = x.shape
        a = alphas.detach().float().contiguous().view(-1)
        im = imp.detach().float().contiguous()
        wf, bf = w.detach().float().contiguous(), b.detach().float().contiguous()
        y = _new_like(vx[0])
        lib.adr_adyt_fwd(dcode(x.dtype), ctypes.c_void_p(vx[1]), vx[2], fptr(a), fptr(im), fptr(wf), fptr(bf),
                         ctypes.c_void_p(y.data_ptr()), C, N, H * W, C, stream())
        ctx.save_for_backward(vx[0], a, im, wf)
        ctx.ashape = alphas.shape
        ctx.params = (alphas, w, b)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, a, im, wf = ctx.saved_tensors
        N, C, H, W = x.shape
        vx, vd = _v(x), _v(dy)
        dev = x.device
        dx = _new_like(x)
        dimp = torch.empty(N, 3, dtype=torch.float32, device=dev)
        da = torch.empty(3, dtype=torch.float32, device=dev)
        dw = torch.empty(C, dtype=torch.float32, device=dev)
        db = torch.empty(C, dtype=torch.float32, device=dev)
        wsb = lib.adr_adyt_bwd_workspace(N, H * W, C)
        ws = torch.empty(wsb // 4 + 1, dtype=torch.float32, device=dev)
        lib.adr_adyt_bwd(dcode(x.dtype), ctypes.c_void_p(vx[1]), vx[2], ctypes.c_void_p(vd[1]), vd[2], fptr(a), fptr(im),
                         fptr(wf), ctypes.c_void_p(dx.data_ptr()), C, fptr(dimp), fptr(da), fptr(dw), fptr(db), N,
                         H * W, C, fptr(ws), wsb, stream())
        pa, pw, pb = ctx.params
        return dx, sink(pa, da.view(ctx.ashape)), dimp, sink(pw, dw), sink(pb, db)


def adyt(x, alphas, imp, w, b):
    return ADyTFn.apply(x, alphas, imp, w, b)


def tokens(x):
    """(B, C, H, W) NHWC -> (B, C, H*W, 1) NHWC token view (same memory)."""
    B, C, H, W = x.shape
    t, _, cs = _v(x)
    if cs != C:
        t = t.contiguous(memory_format=torch.channels_last)
        relayout_count[0] += 1
    # a view (H and W merge: stride W*C = W x C), not as_strided: as_strided's backward zero-fills the base storage
    # and scatters into it (a fill + copy launch per call)
    return t.view(B, C, H * W, 1)


def untokens(t, H, W):
    B, C, N, _ = t.shape
    t, _, cs = _v(t)
    if cs != C:
        t = t.contiguous(memory_format=torch.channels_last)
        relayout_count[0] += 1
    return t.view(B, C, H, W)


class TSSAStackFn(torch.autograd.Function):
    """Per-scale TSSA (block.py:2465-2477) for S scales, written stacked as (B, C, S*N, 1) tokens
    (torch.stack(scale_features, 1).view(B, S*N, C), :2482-2484)."""

    @staticmethod
    def forward(ctx, temps, heads, *qkvs):
        S = len(qkvs)
        B, C3, N, _ = qkvs[0].shape
        C = C3 // 3
        D = C // heads
        dtype = qkvs[0].dtype
        dev = qkvs[0].device
        out = empty_act(B, C, S * N, 1, dtype, dev)
        tf = temps.detach().float().contiguous().view(S, heads)
        Pi = torch.empty(S, B, heads, N, dtype=torch.float32, device=dev)
        ss = torch.empty_like(Pi)
        att = torch.empty(S, B, heads, D, dtype=torch.float32, device=dev)
        es = out.element_size()
        saved = []
        for s, qkv in enumerate(qkvs):
            t, p, cs = _v(qkv)
            saved.append(t)
            lib.adr_tssa_fwd(dcode(dtype), ctypes.c_void_p(p), ctypes.c_void_p(p + C * es), ctypes.c_void_p(p + 2 * C * es),
                             cs, B, N, heads, D, fptr(tf[s]), ctypes.c_void_p(out.data_ptr() + s * N * C * es), C,
                             S * N, fptr(Pi[s]), fptr(ss[s]), fptr(att[s]), stream())
        ctx.save_for_backward(tf, Pi, ss, att, *saved)
        ctx.meta = (heads, temps.shape)
        ctx.pt = temps
        return out

    @staticmethod
    def backward(ctx, dout):
        tf, Pi, ss, att, *qkvs = ctx.saved_tensors
        heads, tshape = ctx.meta
        S = len(qkvs)
        B, C3, N, _ = qkvs[0].shape
        C, D = C3 // 3, C3 // 3 // heads
        dtype = qkvs[0].dtype
        dev = qkvs[0].device
        dd, ddp, dcs = _v(dout)
        es = dd.element_size()
        dtemp = torch.empty(S, heads, dtype=torch.float32, device=dev)
        ws = torch.empty(B * heads, dtype=torch.float32, device=dev)
        grads = []
        for s, qkv in enumerate(qkvs):
            _, p, cs = _v(qkv)
            g = empty_act(B, C3, N, 1, dtype, dev)
            gp = g.data_ptr()
            lib.adr_tssa_bwd(dcode(dtype), ctypes.c_void_p(p), ctypes.c_void_p(p + C * es), ctypes.c_void_p(p + 2 * C * es),
                             cs, B, N, heads, D, fptr(tf[s]), ctypes.c_void_p(ddp + s * N * C * es), dcs, S * N,
                             fptr(Pi[s]), fptr(ss[s]), fptr(att[s]), ctypes.c_void_p(gp), ctypes.c_void_p(gp + C * es),
                             ctypes.c_void_p(gp + 2 * C * es), C3, fptr(dtemp[s]), fptr(ws), stream())
            grads.append(g)
        return (sink(ctx.pt, dtemp.view(tshape)), None, *grads)


def tssa_stack(temps, heads, qkvs):
    return TSSAStackFn.apply(temps, heads, *qkvs)


class AttnFn(torch.autograd.Function):
    """softmax(q k^T / sqrt(d)) v for the packed in_proj output qkv (B, 3E, L, 1) -> (B, E, L, 1)."""

    @staticmethod
    def forward(ctx, qkv, heads):
        t, p, cs = _v(qkv)
        B, C3, L, _ = qkv.shape
        E = C3 // 3
        hd = E // heads
        o = empty_act(B, E, L, 1, qkv.dtype, qkv.device)
        lse = torch.empty(B * heads * L, dtype=torch.float32, device=qkv.device)
        lib.adr_attn_fwd(dcode(qkv.dtype), ctypes.c_void_p(p), ctypes.c_void_p(p), ctypes.c_void_p(p), cs, 0, E, 2 * E,
                         hd, ctypes.c_void_p(o.data_ptr()), E, B, L, heads, hd, hd, float(hd ** -0.5), fptr(lse),
                         stream())
        ctx.save_for_backward(t, o, lse)
        ctx.heads = heads
        return o

    @staticmethod
    def backward(ctx, do):
        t, o, lse = ctx.saved_tensors
        heads = ctx.heads
        _, p, cs = _v(t)
        dd, ddp, dcs = _v(do)
        B, C3, L, _ = t.shape
        E = C3 // 3
        hd = E // heads
        g = empty_act(B, C3, L, 1, t.dtype, t.device)
        dvec = torch.empty(B * heads * L, dtype=torch.float32, device=t.device)
        gp = g.data_ptr()
        lib.adr_attn_bwd(dcode(t.dtype), ctypes.c_void_p(p), ctypes.c_void_p(p), ctypes.c_void_p(p), cs, 0, E, 2 * E,
                         hd, ctypes.c_void_p(o.data_ptr()), E, ctypes.c_void_p(ddp), dcs, fptr(lse),
                         ctypes.c_void_p(gp), ctypes.c_void_p(gp), ctypes.c_void_p(gp), C3, 0, E, 2 * E, B, L, heads,
                         hd, hd, float(hd ** -0.5), fptr(dvec), stream())
        return g, None


def attention(qkv, heads):
    return AttnFn.apply(qkv, heads)


class PSAAttnFn(torch.autograd.Function):
    """The core of C2PSA's Attention (block.py:906-927) on the NHWC qkv activation (B, heads*(2kd+hd), H, W)
    whose channels are per head [q(kd) k(kd) v(hd)] — `qkv.view(B, heads, 2kd+hd, N).split(...)`. Returns
    o = (v @ softmax(q^T k * kd^-0.5)^T).view(B, C, H, W) and v.reshape(B, C, H, W) (the input of `pe`) as NHWC
    activations; backward writes dq/dk/dv straight into one qkv-shaped gradient and adds pe's v-gradient."""

    @staticmethod
    def forward(ctx, qkv, heads, kd, hd):
        ctx.set_materialize_grads(False)
        t, p, cs = _v(qkv)
        B, Ctot, H, W = qkv.shape
        hs = 2 * kd + hd
        if Ctot != heads * hs:
            raise RuntimeError(f"psa_attention: {Ctot} channels != heads {heads} x (2*{kd}+{hd})")
        L, C = H * W, heads * hd
        o = empty_act(B, C, H, W, qkv.dtype, qkv.device)
        lse = torch.empty(B * heads * L, dtype=torch.float32, device=qkv.device)
        lib.adr_attn_fwd(dcode(qkv.dtype), ctypes.c_void_p(p), ctypes.c_void_p(p), ctypes.c_void_p(p), cs, 0, kd,
                         2 * kd, hs, ctypes.c_void_p(o.data_ptr()), C, B, L, heads, kd, hd, float(kd ** -0.5),
                         fptr(lse), stream())
        v = empty_act(B, C, H, W, qkv.dtype, qkv.device)
        for h in range(heads):
            dst = v[:, h * hd:(h + 1) * hd]
            _ew(EW_COPY, (dst, dst.data_ptr(), C), _v(t[:, h * hs + 2 * kd:h * hs + 2 * kd + hd]))
        ctx.save_for_backward(t, o, lse)
        ctx.meta = (heads, kd, hd)
        return o, v

    @staticmethod
    def backward(ctx, do, dv_pe):
        t, o, lse = ctx.saved_tensors
        heads, kd, hd = ctx.meta
        _, p, cs = _v(t)
        B, Ctot, H, W = t.shape
        L, C, hs = H * W, heads * hd, 2 * kd + hd
        g = empty_act(B, Ctot, H, W, t.dtype, t.device)
        gp = g.data_ptr()
        if do is None:
            zero_(g)
        else:
            dd, ddp, dcs = _v(do.to(t.dtype) if do.dtype != t.dtype else do)
            dvec = torch.empty(B * heads * L, dtype=torch.float32, device=t.device)
            lib.adr_attn_bwd(dcode(t.dtype), ctypes.c_void_p(p), ctypes.c_void_p(p), ctypes.c_void_p(p), cs, 0, kd,
                             2 * kd, hs, ctypes.c_void_p(o.data_ptr()), C, ctypes.c_void_p(ddp), dcs, fptr(lse),
                             ctypes.c_void_p(gp), ctypes.c_void_p(gp), ctypes.c_void_p(gp), Ctot, 0, kd, 2 * kd, B, L,
                             heads, kd, hd, float(kd ** -0.5), fptr(dvec), stream())
        if dv_pe is not None:
            dv_pe = _v(dv_pe.to(t.dtype) if dv_pe.dtype != t.dtype else dv_pe)[0]
            for h in range(heads):
                dst = g[:, h * hs + 2 * kd:h * hs + 2 * kd + hd]
                _ew(EW_COPY, (dst, dst.data_ptr(), Ctot), _v(dv_pe[:, h * hd:(h + 1) * hd]), accumulate=1)
        return g, None, None, None


def psa_attention(qkv, heads, kd, hd):
    return PSAAttnFn.apply(qkv, heads, kd, hd)


class GroupMeanFn(torch.autograd.Function):
    """(B, C, S*N, 1) -> mean over the S stacked groups -> (B, C, N, 1)."""

    @staticmethod
    def forward(ctx, x, S):
        t, p, cs = _v(x)
        B, C, SN, _ = x.shape
        N = SN // S
        y = empty_act(B, C, N, 1, x.dtype, x.device)
        lib.adr_group_mean(dcode(x.dtype), ctypes.c_void_p(p), cs, S, N, ctypes.c_void_p(y.data_ptr()), C, B, C, 0,
                           stream())
        ctx.meta = (S, x.shape, x.dtype)
        return y

    @staticmethod
    def backward(ctx, dy):
        S, shape, dtype = ctx.meta
        B, C, SN, _ = shape
        t, p, cs = _v(dy)
        dx = empty_act(B, C, SN, 1, dtype, dy.device)
        lib.adr_group_mean(dcode(dtype), ctypes.c_void_p(p), cs, S, SN // S, ctypes.c_void_p(dx.data_ptr()), C, B, C, 1,
                           stream())
        return dx, None


def group_mean(x, S):
    return GroupMeanFn.apply(x, S)


class AdaPoolFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, oh, ow):
        t, p, cs = _v(x)
        N, C, H, W = x.shape
        y = empty_act(N, C, oh, ow, x.dtype, x.device)
        lib.adr_adapool(dcode(x.dtype), ctypes.c_void_p(p), cs, N, H, W, C, ctypes.c_void_p(y.data_ptr()), C, oh, ow,
                        stream())
        ctx.meta = (x.shape, x.dtype)
        ctx.sink = _sink_of(x)
        return y

    @staticmethod
    def backward(ctx, dy):
        (N, C, H, W), dtype = ctx.meta
        t, p, cs = _v(dy)
        dx, acc = _dx_dst(ctx, (N, C, H, W), dtype, dy.device)
        lib.adr_adapool_bwd(dcode(dtype), ctypes.c_void_p(p), cs, N, H, W, C, ctypes.c_void_p(dx.data_ptr()),
                            dx.stride(3), dy.shape[2], dy.shape[3], acc, stream())
        return (None if ctx.sink is not None else dx), None, None


def adaptive_avg_pool(x, oh, ow):
    return AdaPoolFn.apply(x, oh, ow)


class BilinearFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, oh, ow):
        t, p, cs = _v(x)
        N, C, H, W = x.shape
        y = empty_act(N, C, oh, ow, x.dtype, x.device)
        lib.adr_bilinear(dcode(x.dtype), ctypes.c_void_p(p), cs, N, H, W, C, ctypes.c_void_p(y.data_ptr()), C, oh, ow,
                         stream())
        ctx.meta = (x.shape, x.dtype)
        ctx.sink = _sink_of(x)
        return y

    @staticmethod
    def backward(ctx, dy):
        (N, C, H, W), dtype = ctx.meta
        t, p, cs = _v(dy)
        dx, acc = _dx_dst(ctx, (N, C, H, W), dtype, dy.device)
        lib.adr_bilinear_bwd(dcode(dtype), ctypes.c_void_p(p), cs, N, H, W, C, ctypes.c_void_p(dx.data_ptr()),
                             dx.stride(3), dy.shape[2], dy.shape[3], acc, stream())
        return (None if ctx.sink is not None else dx), None, None


def bilinear(x, oh, ow):
    return BilinearFn.apply(x, oh, ow)


class UpsampleNearestFn(torch.autograd.Function):
    """nn.Upsample(scale_factor=s, mode='nearest') on NHWC; the output may be a caller's concat slice."""

    @staticmethod
    def forward(ctx, x, s, box=None):
        t, p, cs = _v(x)
        N, C, H, W = x.shape
        y, yp, ycs = _out_view(box, N, C, H * s, W * s, x.dtype, x.device)
        lib.adr_upsample_nearest(dcode(x.dtype), ctypes.c_void_p(p), cs, N, H, W, C, ctypes.c_void_p(yp), ycs, s,
                                 stream())
        ctx.meta = (x.shape, x.dtype, s)
        ctx.sink = _sink_of(x)
        return y if box is None else y[:, :]

    @staticmethod
    def backward(ctx, dy):
        (N, C, H, W), dtype, s = ctx.meta
        t, p, cs = _v(dy.to(dtype) if dy.dtype != dtype else dy)
        dx, acc = _dx_dst(ctx, (N, C, H, W), dtype, dy.device)
        lib.adr_upsample_nearest_bwd(dcode(dtype), ctypes.c_void_p(p), cs, N, H, W, C, ctypes.c_void_p(dx.data_ptr()),
                                     dx.stride(3), s, acc, stream())
        return (None if ctx.sink is not None else dx), None, None


def upsample_nearest(x, s, out=None):
    return UpsampleNearestFn.apply(x, int(s), None if out is None else OutBox(out))


_EDFFN_BASIS = {}


def edffn_basis(device, ps=8):
    """B[uv][i][j] = (irfft2(e_uv * rfft2(e_j)))_i for the 8x8 patch, (8 x 5) half spectrum, float64 host
    construction (numpy pocketfft, the same C2R convention torch.fft uses) -> fp32 device constant."""
    key = (str(device), ps)
    if key not in _EDFFN_BASIS:
        import numpy as np
        nv = ps // 2 + 1
        eye = np.eye(ps * ps).reshape(ps * ps, ps, ps)
        spec = np.fft.rfft2(eye)
        B = np.empty((ps * nv, ps * ps, ps * ps))
        for u in range(ps):
            for v in range(nv):
                filt = np.zeros((ps, nv))
                filt[u, v] = 1.0
                y = np.fft.irfft2(spec * filt, s=(ps, ps)).reshape(ps * ps, ps * ps)  # [j][i]
                B[u * nv + v] = y.T
        _EDFFN_BASIS[key] = torch.from_numpy(B.astype(np.float32)).to(device)
    return _EDFFN_BASIS[key]


class EDFFNFilterFn(torch.autograd.Function):
    """Reflect-pad to a multiple of 8, per-patch rfft2 * fft -> irfft2, crop (block.py:2399-2413)."""

    @staticmethod
    def forward(ctx, x, fft):
        t, p, cs = _v(x)
        N, C, H, W = x.shape
        basis = edffn_basis(x.device)
        wf = fft.detach().float().contiguous().view(C, -1)
        M = torch.empty(C, 64, 64, dtype=torch.float32, device=x.device)
        lib.adr_edffn_build(fptr(wf), fptr(basis), C, wf.shape[1], fptr(M), stream())
        y = empty_act(N, C, H, W, x.dtype, x.device)
        lib.adr_edffn_fwd(dcode(x.dtype), ctypes.c_void_p(p), cs, fptr(M), ctypes.c_void_p(y.data_ptr()), C, N, H, W, C,
                          stream())
        ctx.save_for_backward(t, M)
        ctx.meta = (fft.shape, wf.shape[1])
        ctx.pf = fft
        return y

    @staticmethod
    def backward(ctx, dy):
        t, M = ctx.saved_tensors
        fshape, nuv = ctx.meta
        N, C, H, W = t.shape
        _, p, cs = _v(t)
        dd, dp, dcs = _v(dy)
        basis = edffn_basis(t.device)
        dx = empty_act(N, C, H, W, t.dtype, t.device)
        dw, pdw, acc = grad_dst(ctx.pf, C * nuv, t.device)
        wsb = lib.adr_edffn_bwd_workspace(N, H, W, C)
        ws = torch.empty(wsb // 4 + 1, dtype=torch.float32, device=t.device)
        lib.adr_edffn_bwd(dcode(t.dtype), ctypes.c_void_p(p), cs, ctypes.c_void_p(dp), dcs, fptr(M), fptr(basis), nuv,
                          ctypes.c_void_p(dx.data_ptr()), C, pdw, N, H, W, C, acc, fptr(ws), wsb, stream())
        return dx, grad_ret(ctx.pf, dw)


def edffn_filter(x, fft):
    return EDFFNFilterFn.apply(x, fft)


# ------------------------------------------------------------------------------------------------------------
# 697 L10 variant: DynamicTanh, Mona norm-mix, AttentionTSSA core, dropout (adr_mona.hip)
# ------------------------------------------------------------------------------------------------------------


def _f32(t):
    return t.detach().float().contiguous()


class DyTFn(torch.autograd.Function):
    """DynamicTanh (block.py:1624-1641, channels_first): tanh(alpha x) * w[c] + b[c]."""

    @staticmethod
    def forward(ctx, x, alpha, w, b):
        vx = _v(x)
        N, C, H, W = x.shape
        af, wf, bf = _f32(alpha), _f32(w), _f32(b)
        y = _new_like(vx[0])
        lib.adr_dyt_fwd(dcode(x.dtype), ctypes.c_void_p(vx[1]), vx[2], fptr(af), fptr(wf), fptr(bf),
                        ctypes.c_void_p(y.data_ptr()), C, N * H * W, C, stream())
        ctx.save_for_backward(vx[0], af, wf)
        ctx.params = (alpha, w, b)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, af, wf = ctx.saved_tensors
        pa, pw, pb = ctx.params
        N, C, H, W = x.shape
        vx, vd = _v(x), _v(dy.to(x.dtype) if dy.dtype != x.dtype else dy)
        dev = x.device
        dx = _new_like(x)
        # the three parameter gradients share one destination kind (all in the arena, or all fresh)
        da, pda, acc = grad_dst(pa, 1, dev)
        dw, pdw, acc_w = grad_dst(pw, C, dev)
        db, pdb, acc_b = grad_dst(pb, C, dev)
        if not acc == acc_w == acc_b:
            raise RuntimeError("DynamicTanh parameter gradients must share one destination kind")
        wsb = lib.adr_dyt_bwd_workspace(N * H * W, C)
        ws = torch.empty(wsb // 4 + 1, dtype=torch.float32, device=dev)
        lib.adr_dyt_bwd(dcode(x.dtype), ctypes.c_void_p(vx[1]), vx[2], ctypes.c_void_p(vd[1]), vd[2], fptr(af),
                        fptr(wf), ctypes.c_void_p(dx.data_ptr()), C, pda, pdw, pdb, acc, N * H * W, C, fptr(ws), wsb,
                        stream())
        return dx, grad_ret(pa, da), grad_ret(pw, dw), grad_ret(pb, db)


def dyt(x, alpha, w, b):
    return DyTFn.apply(x, alpha, w, b)


class LnMixFn(torch.autograd.Function):
    """Mona prologue (mona.py:5-10, 55-58): LayerNorm2d(x) * gamma + x * gammax (LayerNorm over channels)."""

    @staticmethod
    def forward(ctx, x, lw, lb, gamma, gammax, eps):
        vx = _v(x)
        N, C, H, W = x.shape
        dev = x.device
        ps = [_f32(p).view(-1) for p in (lw, lb, gamma, gammax)]
        y = _new_like(vx[0])
        mean = torch.empty(N * H * W, dtype=torch.float32, device=dev)
        rstd = torch.empty_like(mean)
        lib.adr_ln_mix_fwd(dcode(x.dtype), ctypes.c_void_p(vx[1]), vx[2], *[fptr(p) for p in ps],
                           ctypes.c_void_p(y.data_ptr()), C, fptr(mean), fptr(rstd), N * H * W, C, float(eps),
                           stream())
        ctx.save_for_backward(vx[0], *ps, mean, rstd)
        ctx.params = (lw, lb, gamma, gammax)
        return y

    @staticmethod
    def backward(ctx, dz):
        x, lw, lb, gm, gx, mean, rstd = ctx.saved_tensors
        N, C, H, W = x.shape
        dev = x.device
        vx, vd = _v(x), _v(dz.to(x.dtype) if dz.dtype != x.dtype else dz)
        dx = _new_like(x)
        dsts = [grad_dst(p, C, dev) for p in ctx.params]
        if len({d[2] for d in dsts}) != 1:
            raise RuntimeError("Mona norm parameter gradients must share one destination kind")
        wsb = lib.adr_ln_mix_bwd_workspace(N * H * W, C)
        ws = torch.empty(wsb // 4 + 1, dtype=torch.float32, device=dev)
        lib.adr_ln_mix_bwd(dcode(x.dtype), ctypes.c_void_p(vx[1]), vx[2], ctypes.c_void_p(vd[1]), vd[2], fptr(lw),
                           fptr(lb), fptr(gm), fptr(gx), fptr(mean), fptr(rstd), ctypes.c_void_p(dx.data_ptr()), C,
                           *[d[1] for d in dsts], dsts[0][2], N * H * W, C, fptr(ws), wsb, stream())
        return (dx, *[grad_ret(p, d[0]) for p, d in zip(ctx.params, dsts)], None)


def ln_mix(x, lw, lb, gamma, gammax, eps=1e-5):
    return LnMixFn.apply(x, lw, lb, gamma, gammax, eps)


class TSSA1Fn(torch.autograd.Function):
    """AttentionTSSA core (block.py:1655-1683) on (B, C, N, 1) token tensors: w -> -w * Pi * attn."""

    @staticmethod
    def forward(ctx, w, temp, heads):
        t, p, cs = _v(w)
        B, C, N, _ = w.shape
        D = C // heads
        dev = w.device
        tf = _f32(temp).view(-1)
        state = torch.empty(lib.adr_tssa1_state_floats(B, N, heads, D), dtype=torch.float32, device=dev)
        out = empty_act(B, C, N, 1, w.dtype, dev)
        lib.adr_tssa1_fwd(dcode(w.dtype), ctypes.c_void_p(p), cs, B, N, heads, D, fptr(tf),
                          ctypes.c_void_p(out.data_ptr()), C, fptr(state), stream())
        ctx.save_for_backward(t, tf, state)
        ctx.meta = heads
        ctx.pt = temp
        return out

    @staticmethod
    def backward(ctx, dout):
        t, tf, state = ctx.saved_tensors
        heads = ctx.meta
        B, C, N, _ = t.shape
        D = C // heads
        dev = t.device
        _, p, cs = _v(t)
        _, gp, gcs = _v(dout.to(t.dtype) if dout.dtype != t.dtype else dout)
        dw = empty_act(B, C, N, 1, t.dtype, dev)
        dtemp, pdt, acc = grad_dst(ctx.pt, heads, dev)
        wsb = lib.adr_tssa1_bwd_workspace(B, N, heads, D)
        ws = torch.empty(wsb // 4 + 1, dtype=torch.float32, device=dev)
        lib.adr_tssa1_bwd(dcode(t.dtype), ctypes.c_void_p(p), cs, B, N, heads, D, fptr(tf), fptr(state),
                          ctypes.c_void_p(gp), gcs, ctypes.c_void_p(dw.data_ptr()), C, pdt, acc, fptr(ws), wsb,
                          stream())
        return dw, grad_ret(ctx.pt, dtemp), None


def tssa1(w, temp, heads):
    return TSSA1Fn.apply(w, temp, heads)


class DropoutFn(torch.autograd.Function):
    """Inverted dropout with a hash mask keyed by a device seed (advanced on the device after each use, so a
    captured graph draws a new mask per replay); the backward re-derives the same mask."""

    @staticmethod
    def forward(ctx, x, p, seed):
        vx = _v(x)
        N, C, H, W = x.shape
        y = _new_like(vx[0])
        snap = seed.clone()  # this call's seed, for the backward
        lib.adr_dropout(dcode(x.dtype), ctypes.c_void_p(vx[1]), vx[2], ctypes.c_void_p(y.data_ptr()), C, N * H * W, C,
                        float(p), ctypes.c_void_p(snap.data_ptr()), stream())
        lib.adr_seed_advance(ctypes.c_void_p(seed.data_ptr()), stream())
        ctx.save_for_backward(snap)
        ctx.p = p
        return y

    @staticmethod
    def backward(ctx, dy):
        (snap,) = ctx.saved_tensors
        vd = _v(dy)
        N, C, H, W = dy.shape
        dx = _new_like(vd[0])
        lib.adr_dropout(dcode(dy.dtype), ctypes.c_void_p(vd[1]), vd[2], ctypes.c_void_p(dx.data_ptr()), C, N * H * W,
                        C, float(ctx.p), ctypes.c_void_p(snap.data_ptr()), stream())
        return dx, None, None


def dropout(x, p, seed, training):
    if not training or p == 0.0:
        return x
    return DropoutFn.apply(x, p, seed)


# ------------------------------------------------------------------------------------------------------------
# Level-packed AYHead. The reference runs the head once per pyramid level (head.py:1132-1176): ~60 launches per
# level forward, twice that backward, most of them per-pixel kernels that at P4 (40x40) and P5 (20x20) fill a
# fraction of the chip. Here the three levels live in ONE row space — level l's NHWC rows (image, y, x) stored
# back to back, P3 first — so every per-pixel op (1x1 convs, gates, elementwise, activations) is one launch over
# all levels; ops that need the level structure take a LevelPack:
#   * per-image statistics (GroupNorm, the global average pool): the row space is cut into sub-images of S rows
#     (S = gcd of the levels' H*W, the P5 map) and segment kernels combine an image's sub-images
#     (adr_gn_finalize_packed / adr_gn_bwd_coef_packed / adr_seg_mean_packed);
#   * spatial ops (3x3 convs, DCN, CoordAtt's axis means / gates): one launch per level on the level's view, the
#     levels' split-K WGRAD slabs reduced by one entry.
# ------------------------------------------------------------------------------------------------------------
class LevelPack:
    """Geometry of the packed row space: N images per level, level dims [(H, W)]; a packed activation is an
    (N', C, 1, S) NHWC tensor with N' = N * sum(k), k[l] = H_l*W_l / S sub-images per image of level l."""

    def __init__(self, N, dims):
        import math
        self.N = int(N)
        self.dims = tuple((int(h), int(w)) for h, w in dims)
        hw = [h * w for h, w in self.dims]
        S = 0
        for v in hw:
            S = math.gcd(S, v)
        self.S = S
        self.L = len(hw)
        self.k = tuple(v // S for v in hw)
        self.Np = self.N * sum(self.k)
        self.off, o = [], 0
        for v in hw:
            self.off.append(o)
            o += self.N * v
        self.rows = o
        self.sub0 = [off // S for off in self.off]
        self.k_c = (ctypes.c_int * self.L)(*self.k)

    def empty(self, C, dtype, dev):
        return empty_act(self.Np, C, 1, self.S, dtype, dev)

    def fits(self, t):
        return t.shape[0] == self.Np and t.shape[2] == 1 and t.shape[3] == self.S

    def view(self, t, l):
        """Level l of packed t (a whole packed activation or a channel slice of one) as an (N, C, H, W) NHWC view."""
        H, W = self.dims[l]
        C, cs = t.shape[1], t.stride(3)
        return torch.as_strided(t, (self.N, C, H, W), (H * W * cs, 1, W * cs, cs),
                                t.storage_offset() + self.off[l] * cs)

    def at(self, ptr, cs, es, l):
        """Address of level l's first row in a packed buffer at ptr with channel stride cs."""
        return ctypes.c_void_p(ptr + self.off[l] * cs * es)


def _ptrs(ts):
    arr = (ctypes.c_void_p * len(ts))(*[None if t is None else t.data_ptr() for t in ts])
    return ctypes.cast(arr, ctypes.c_void_p), arr


class LevelJoinFn(torch.autograd.Function):
    """Per-level pieces (N, C, H_l, W_l) -> one packed activation. Pieces already written in place through their
    level view of the box (conv2d out=) are not copied. Backward: each piece gets its level view of the gradient."""

    @staticmethod
    def forward(ctx, box, pack, *xs):
        x0 = xs[0]
        C = x0.shape[1]
        out = pack.empty(C, x0.dtype, x0.device) if box is None else box.t
        if not pack.fits(out) or out.shape[1] != C:
            raise RuntimeError("level_join: out must be a packed activation of the pieces' channels")
        for l, x in enumerate(xs):
            o = pack.view(out, l)
            v = _v(x)
            if not (v[1] == o.data_ptr() and v[2] == o.stride(3)):
                _ew(EW_COPY, (o, o.data_ptr(), o.stride(3)), v)
        ctx.pack = pack
        return out if box is None else out[:, :]

    @staticmethod
    def backward(ctx, dy):
        dy, _, _ = _v(dy)
        return (None, None) + tuple(ctx.pack.view(dy, l) for l in range(ctx.pack.L))


def level_join(xs, pack, out=None):
    return LevelJoinFn.apply(None if out is None else OutBox(out), pack, *xs)


class LevelSplitFn(torch.autograd.Function):
    """Packed activation -> its per-level (N, C, H_l, W_l) views (the head's output list). Backward: gradients that
    are the level views of one packed buffer (the loss writes them so) are handed back as that buffer."""

    @staticmethod
    def forward(ctx, x, pack):
        ctx.set_materialize_grads(False)
        ctx.pack, ctx.meta = pack, (tuple(x.shape), x.dtype)
        return tuple(pack.view(x, l) for l in range(pack.L))

    @staticmethod
    def backward(ctx, *grads):
        pack = ctx.pack
        (Np, C, _, S), dtype = ctx.meta
        if all(g is not None and g.dtype == dtype for g in grads):
            g0 = grads[0]
            cs, es, st = g0.stride(3), g0.element_size(), g0.untyped_storage().data_ptr()
            ok = cs >= C and cs % (16 // es) == 0
            for l, g in enumerate(grads):
                H, W = pack.dims[l]
                ok = ok and g.untyped_storage().data_ptr() == st and \
                    g.stride() == (H * W * cs, 1, W * cs, cs) and \
                    g.data_ptr() == g0.data_ptr() + (pack.off[l] - pack.off[0]) * cs * es
            if ok:
                return torch.as_strided(g0, (Np, C, 1, S), (S * cs, 1, S * cs, cs), g0.storage_offset()), None
        dev = next(g for g in grads if g is not None).device
        dx = pack.empty(C, dtype, dev)
        es = dx.element_size()
        for l, g in enumerate(grads):
            o = pack.view(dx, l)
            if g is None:
                lib.adr_memset_zero(ctypes.c_void_p(o.data_ptr()), o.numel() * es, stream())
            else:
                _ew(EW_COPY, (o, o.data_ptr(), C), _v(g.to(dtype) if g.dtype != dtype else g))
        return dx, None


def level_split(x, pack):
    outs = LevelSplitFn.apply(x, pack)
    for o in outs:
        o._adr_pack = pack
    return outs


class GNPackFn(torch.autograd.Function):
    """act(GroupNorm(G)(y)) per (level, image) of a packed activation: nc_reduce over the sub-images, one segmented
    finalize, affine_act with per-sub-image coefficients; backward the same three launches. `params` holds
    (gamma, beta) of a GroupNorm shared by the levels, or per_level: gamma_0..gamma_{L-1}, beta_0..beta_{L-1}."""

    @staticmethod
    def forward(ctx, y, pack, groups, act, eps, per_level, *params):
        dtype = y.dtype
        ctx.gate, ctx.eps = getattr(y, "_adr_gate", None) if _GN_GATE else None, eps  # y = s*conv() (ScaleFn)
        y, yp, ycs = nhwc(y)
        Np, C, _, S = y.shape
        dev = y.device
        nl = len(params) // 2
        gam = [params[l if per_level else 0].detach() for l in range(pack.L)]
        bet = [params[nl + (l if per_level else 0)].detach() for l in range(pack.L)]
        rows = _stats_rows(Np, S)
        chunks = lib.adr_nc_reduce_chunks(S, rows)
        part = torch.empty(Np * chunks * 2 * C, dtype=torch.float32, device=dev)
        scale = torch.empty(Np * C, dtype=torch.float32, device=dev)
        shift = torch.empty(Np * C, dtype=torch.float32, device=dev)
        mean = torch.empty(Np * groups, dtype=torch.float32, device=dev)
        rstd = torch.empty(Np * groups, dtype=torch.float32, device=dev)
        lib.adr_nc_reduce(dcode(dtype), 0, ctypes.c_void_p(yp), ycs, 0, None, 0, 0, None, None, 0, 0, Np, S, C, rows,
                          fptr(part), stream())
        (gp, _ga), (bp, _ba) = _ptrs(gam), _ptrs(bet)
        lib.adr_gn_finalize_packed(fptr(part), pack.L, ctypes.cast(pack.k_c, ctypes.c_void_p), pack.N, chunks, S, C,
                                   groups, gp, bp, float(eps), fptr(scale), fptr(shift), fptr(mean), fptr(rstd),
                                   stream())
        z = pack.empty(C, dtype, dev)
        lib.adr_affine_act(dcode(dtype), ctypes.c_void_p(yp), ycs, 0, ctypes.c_void_p(z.data_ptr()), C, 0,
                           fptr(scale), fptr(shift), 1, ACT[act], Np, S, C, stream())
        ctx.save_for_backward(y, scale, shift, mean, rstd)
        ctx.meta = (groups, act, bool(per_level), chunks, rows)
        ctx.pack, ctx.params = pack, params
        return z

    @staticmethod
    def backward(ctx, dz):
        y, scale, shift, mean, rstd = ctx.saved_tensors
        groups, act, per_level, chunks, rows = ctx.meta
        pack, params = ctx.pack, ctx.params
        dz, dzp, dzcs = nhwc(dz.to(y.dtype) if dz.dtype != y.dtype else dz)
        _, yp, ycs = nhwc(y)
        Np, C, _, S = y.shape
        dev = y.device
        dt = dcode(y.dtype)
        nl = len(params) // 2
        part = torch.empty(Np * chunks * 2 * C, dtype=torch.float32, device=dev)
        lib.adr_nc_reduce(dt, 1, ctypes.c_void_p(yp), ycs, 0, ctypes.c_void_p(dzp), dzcs, 0, fptr(scale),
                          fptr(shift), 1, ACT[act], Np, S, C, rows, fptr(part), stream())
        A = torch.empty(Np * C, dtype=torch.float32, device=dev)
        B = torch.empty(Np * C, dtype=torch.float32, device=dev)
        Cc = torch.empty(Np * C, dtype=torch.float32, device=dev)
        gp, _ga = _ptrs([params[l if per_level else 0].detach() for l in range(pack.L)])
        lib.adr_gn_bwd_coef_packed(fptr(part), pack.L, ctypes.cast(pack.k_c, ctypes.c_void_p), pack.N, chunks, S, C,
                                   groups, gp, fptr(mean), fptr(rstd), fptr(A), fptr(B), fptr(Cc), stream())
        dy = pack.empty(C, y.dtype, dev)
        lib.adr_affine_act_bwd(dt, ctypes.c_void_p(yp), ycs, 0, ctypes.c_void_p(dzp), dzcs, 0,
                               ctypes.c_void_p(dy.data_ptr()), C, 0, fptr(scale), fptr(shift), fptr(A), fptr(B),
                               fptr(Cc), 1, 1, ACT[act], Np, S, C, 0, stream())
        if ctx.gate is not None:
            _gn_gate_grad(ctx.gate, ctx.eps, part, list(pack.k), pack.N, chunks, S, C, groups,
                          [params[l if per_level else 0].detach() for l in range(pack.L)], mean, rstd, dy)
        grads = [None] * len(params)
        for j in range(nl):  # dgamma / dbeta over the sub-images of level j (or of every level: shared)
            s0, n = (pack.sub0[j], pack.N * pack.k[j]) if per_level else (0, Np)
            pv, mv, rv = part[s0 * chunks * 2 * C:], mean[s0 * groups:], rstd[s0 * groups:]
            gam, bet = params[j], params[nl + j]
            dgamma, pg, acc_g = grad_dst(gam, C, dev)
            dbeta, pb, acc_b = grad_dst(bet, C, dev)
            if acc_g != acc_b:
                raise RuntimeError("GN gamma/beta gradients must share one destination kind")
            if _defer_gn(acc_g):
                _dfr().add_gnparam(pv, mv, rv, pg, pb, n, chunks, C, groups, acc_g)
            else:
                val = lambda q: q.value if isinstance(q, ctypes.c_void_p) else q  # noqa: E731
                arr = (GnParamEntry * 1)(GnParamEntry(pv.data_ptr(), mv.data_ptr(), rv.data_ptr(), val(pg), val(pb),
                                                      n, chunks, C, groups, acc_g, 0))
                lib.adr_gn_param_grad_batched(ctypes.cast(arr, ctypes.c_void_p), 1, stream())
            grads[j], grads[nl + j] = grad_ret(gam, dgamma), grad_ret(bet, dbeta)
        return (dy, None, None, None, None, None, *grads)


def gn_act_packed(y, pack, gns, act):
    """GroupNorm + activation of a packed activation; gns: one nn.GroupNorm shared by the levels, or one per level."""
    gns = list(gns)
    per_level = len(gns) > 1
    if per_level and len(gns) != pack.L:
        raise RuntimeError("gn_act_packed: one GroupNorm, or one per level")
    g0 = gns[0]
    return GNPackFn.apply(y, pack, g0.num_groups, act, g0.eps, per_level, *[g.weight for g in gns],
                          *[g.bias for g in gns])


def _seg(inp, in_seg, out_seg, mean, pack, C):
    """adr_seg_reduce_packed over fp32 rows of C: per (level, image) segment <-> per sub-image."""
    rows = pack.L * pack.N if out_seg else pack.Np
    out = torch.empty(rows, C, dtype=torch.float32, device=inp.device)
    lib.adr_seg_reduce_packed(fptr(inp), int(in_seg), int(out_seg), int(mean), pack.L,
                              ctypes.cast(pack.k_c, ctypes.c_void_p), pack.N, pack.S, C, fptr(out), stream())
    return out


class GapPackFn(torch.autograd.Function):
    """Global average pool per (level, image) of a packed activation: (L * N, C) fp32, level-major
    (F.adaptive_avg_pool2d(x, 1), head.py:1142, for every level at once)."""

    @staticmethod
    def forward(ctx, x, pack):
        Np, C, _, S = x.shape
        s = _reduce_dot(None, x, False, False, which=1)  # per-sub-image sums
        ctx.pack, ctx.meta = pack, (tuple(x.shape), x.dtype)
        ctx.sink = _sink_of(x)
        return _seg(s, False, True, True, pack, C)

    @staticmethod
    def backward(ctx, dg):
        pack = ctx.pack
        (Np, C, _, S), dtype = ctx.meta
        t = _seg(dg.float().contiguous(), True, False, True, pack, C)
        dx, acc = _dx_dst(ctx, (Np, C, 1, S), dtype, dg.device)
        lib.adr_bcast_fill(dcode(dtype), fptr(t), C, 1, 1.0, ctypes.c_void_p(dx.data_ptr()), dx.stride(3), Np, S, C, acc,
                           stream())
        return (None if ctx.sink is not None else dx), None


def gap_packed(x, pack):
    return GapPackFn.apply(x, pack)


class SegExpandFn(torch.autograd.Function):
    """A per-(level, image) vector (L * N,) or rows (L * N, C) -> one copy per sub-image (N', ...): the packed head's
    per-image gates for scale(..., "n"); backward sums the sub-images' gradients."""

    @staticmethod
    def forward(ctx, v, pack):
        C = v.numel() // (pack.L * pack.N)
        ctx.pack, ctx.meta = pack, (tuple(v.shape), C)
        out = _seg(v.detach().float().contiguous(), True, False, False, pack, C)
        return out.view(pack.Np) if v.dim() == 1 else out

    @staticmethod
    def backward(ctx, g):
        shape, C = ctx.meta
        return _seg(g.float().contiguous(), False, True, False, ctx.pack, C).view(shape), None


def seg_expand(v, pack):
    return SegExpandFn.apply(v, pack)


def wgrad_param_multi(param, pieces, K, C, RS, wshape, cpad, device, bias=None):
    """wgrad_param over several contractions of one weight (the head's per-level convs): every piece's split-K slabs
    go to one buffer and ONE reduction sums them all (one deferral entry, no flush for a repeated destination).
    bias: as in wgrad_param — returns (dw, fused, db), the pieces' bias column sums written by the same launches
    (adr_conv2d_wgrad_partials_bias) into one [sum of splits][2][K] row set."""
    K_, C_ = wshape[0], wshape[1]
    RS_ = 1
    for v in wshape[2:]:
        RS_ *= v
    stride = K * RS * C
    splits = [lib.adr_conv2d_wgrad_splits(ctypes.byref(d)) for d, _, _ in pieces]
    ws = torch.empty(sum(splits) * stride, dtype=torch.float32, device=device)
    bpart = None
    if (bias is not None and K == K_ and _fuse_wg_bias() and
            all(lib.adr_conv2d_wgrad_bias_fusable(ctypes.byref(d)) for d, _, _ in pieces)):
        bpart = torch.empty(sum(splits) * 2 * K, dtype=torch.float32, device=device)
    s0 = 0
    for (d, xp, dyp), sp in zip(pieces, splits):
        es = 2 if d.dtype == BF16 else 4
        name = (f"void adr::wgrad_bf16_kernel<{_bn_of(K)}, {_bn_of(C)}>(adr::WgArgs)" if d.dtype == BF16
                else _gemm_symbol(F32, _bn_of(C), 2))
        work = (es * (d.n * d.h * d.w * d.c + d.n * d.ho * d.wo * d.k) + 4 * sp * stride,
                2 * d.n * d.ho * d.wo * d.k * RS * d.c)
        tok = _t0(name, *work, _shape(d, f"wgrad/{sp}") if _TIMING is not None else "")
        if bpart is not None:
            lib.adr_conv2d_wgrad_partials_bias(ctypes.byref(d), ctypes.c_void_p(xp), ctypes.c_void_p(dyp),
                                               ctypes.c_void_p(ws.data_ptr() + 4 * s0 * stride),
                                               ctypes.c_void_p(bpart.data_ptr() + 4 * s0 * 2 * K), stream())
        else:
            lib.adr_conv2d_wgrad_partials(ctypes.byref(d), ctypes.c_void_p(xp), ctypes.c_void_p(dyp),
                                          ctypes.c_void_p(ws.data_ptr() + 4 * s0 * stride), 0, stream())
        _t1(tok)
        s0 += sp
    Cp = max(C_, cpad)
    out, ptr, acc = grad_dst(param, K_ * C_ * RS_, device)
    if _dfr() is not None and acc and _TIMING is None and s0 * stride * 4 <= DEFER_MAX_BYTES:
        _dfr().add(ws, stride, s0, ptr, K_, C_, Cp, RS_, 0, acc)
    else:
        lib.adr_wgrad_reduce_unpack(fptr(ws), stride, s0, ptr, K_, C_, Cp, RS_, 0, acc, stream())
    if bias is None:
        return grad_ret(param, out)
    db = _bias_rows(bias, K, s0, bpart, device) if bpart is not None else None
    return grad_ret(param, out), bpart is not None, db


class LevelConvFn(torch.autograd.Function):
    """Dense stride-1 k x k conv (pad k//2) of a packed activation, level by level (each level's map is its own
    image grid): one launch per level forward and data gradient, the levels' WGRAD slabs reduced once. kpad > 0:
    output channels zero-padded to kpad (PaddedConvFn: 27 -> 32 offsets/mask, 1 -> 8 cls_prob)."""

    @staticmethod
    def forward(ctx, x, w, b, pad, kpad, pack):
        sink_ = getattr(x, "_adr_sink", None)
        ctx.sink = sink_ if sink_ is not None and sink_.fits(x) else None
        dtype = x.dtype
        x, xp, xcs = nhwc(x)
        Np, C, _, S = x.shape
        K, Cw, R, Sk = w.shape
        if Cw != C or not pack.fits(x):
            raise RuntimeError(f"level_conv: input {tuple(x.shape)} vs weight {tuple(w.shape)} / pack")
        dev = x.device
        Kp = max(K, kpad)
        if kpad and dtype != torch.bfloat16:
            wp, wt = torch.empty(Kp * R * Sk * C, dtype=dtype, device=dev), None
            zero_(wp)
            lib.adr_pack_weight(dcode(dtype), fptr(w.detach().float().contiguous()), fptr(wp), K, C, C, R * Sk, 0,
                                stream())
        else:
            wp, wt = pack_weight2(w, dtype, kpad=kpad)
        if kpad:
            bp = _padded_bias(b, K, kpad, dev)
        else:
            bp = b.detach().float().contiguous() if b is not None else None
        y = pack.empty(Kp, dtype, dev)
        es = x.element_size()
        for l, (H, W) in enumerate(pack.dims):
            d, _, _ = conv_desc(pack.N, H, W, C, xcs, Kp, R, Sk, 1, 1, pad, pad, Kp, dtype)
            conv_fwd(d, pack.at(xp, xcs, es, l).value, wp.data_ptr(), fptr(bp), pack.at(y.data_ptr(), Kp, es, l).value)
        ctx.save_for_backward(x, wp, wt)
        ctx.meta = (pad, kpad, tuple(w.shape), b is not None)
        ctx.pw, ctx.pb, ctx.pack = w, b, pack
        return y

    @staticmethod
    def backward(ctx, dy):
        x, wp, wt = ctx.saved_tensors
        pad, kpad, wshape, has_b = ctx.meta
        pack = ctx.pack
        dy, dyp, dycs = nhwc(dy.to(x.dtype) if dy.dtype != x.dtype else dy)
        Np, C, _, S = x.shape
        K, _, R, Sk = wshape
        Kp = max(K, kpad)
        x, xp, xcs = nhwc(x)
        es = x.element_size()
        dev = x.device
        dx = dw = db = None
        if ctx.needs_input_grad[0]:
            if ctx.sink is not None:  # into the fan-out's shared gradient (accumulating after the first consumer)
                buf, acc, _ = ctx.sink.claim(dev)
            else:
                buf, acc = pack.empty(C, x.dtype, dev), 0
            bcs = buf.stride(3)
            for l, (H, W) in enumerate(pack.dims):
                d2, _, _ = conv_desc(pack.N, H, W, C, bcs, Kp, R, Sk, 1, 1, pad, pad, dycs, x.dtype)
                conv_dgrad(d2, pack.at(dyp, dycs, es, l).value, (wp, wt), None, pack.at(buf.data_ptr(), bcs, es, l).value,
                           accumulate=acc)
            dx = None if ctx.sink is not None else buf
        if ctx.needs_input_grad[1]:
            pieces = []
            for l, (H, W) in enumerate(pack.dims):
                d, _, _ = conv_desc(pack.N, H, W, C, xcs, Kp, R, Sk, 1, 1, pad, pad, dycs, x.dtype)
                pieces.append((d, pack.at(xp, xcs, es, l).value, pack.at(dyp, dycs, es, l).value))
            if has_b and ctx.needs_input_grad[2] and not kpad:
                dw, fused, db = wgrad_param_multi(ctx.pw, pieces, Kp, C, R * Sk, wshape, 0, dev, bias=ctx.pb)
            else:
                dw, fused = wgrad_param_multi(ctx.pw, pieces, Kp, C, R * Sk, wshape, 0, dev), False
        else:
            fused = False
        if has_b and ctx.needs_input_grad[2] and not fused:
            if kpad:
                db = sink(ctx.pb, _bias_grad(dy, Kp, Np, S, dycs)[:K])
            else:
                db = _bias_grad(dy, K, Np, S, dycs, ctx.pb)
        return dx, dw, db, None, None, None


def level_conv(x, w, b, pad, pack, kpad=0):
    return LevelConvFn.apply(x, w, b, pad, kpad, pack)


class LevelDCNFn(torch.autograd.Function):
    """DCNFn (mmcv ModulatedDeformConv2d 3x3, head.py:751-782) on a packed activation, level by level; the fp32
    path's column GEMMs run once over every level's rows."""

    @staticmethod
    def forward(ctx, x, om, w, pack):
        dtype = x.dtype
        x, xp, xcs = nhwc(x)
        om, omp, omcs = nhwc(om)
        Np, C, _, S = x.shape
        Cout = w.shape[0]
        dev = x.device
        es = x.element_size()
        N = pack.N
        y = pack.empty(Cout, dtype, dev)
        ctx.fused = _dcn_fused(dtype, C, Cout, omcs)
        ctx.fused_bwd = ctx.fused and C == Cout and C in (64, 128, 256)
        if ctx.fused and DCN_LEVELS and len(pack.dims) <= 3:
            wp = pack_weight2(w, dtype)[0]
            lv = (DcnLevelStruct * len(pack.dims))()
            for l, (H, W) in enumerate(pack.dims):
                lv[l].x, lv[l].om = pack.at(xp, xcs, es, l), pack.at(omp, omcs, es, l)
                lv[l].y = pack.at(y.data_ptr(), Cout, es, l)
                lv[l].H, lv[l].W = H, W
            work = [sum(v) for v in zip(*[_dcn_work(N, H, W, C, Cout) for H, W in pack.dims])]
            tok = _t0("adr::dcn_fwd_levels_kernel(adr::DcnLevels)", *work,
                      f"dcn fwd levels n{N} {pack.dims} c{C}->{Cout}" if _TIMING is not None else "", _reps())
            for _ in range(_reps()):
                lib.adr_dcn_fwd_bf16_levels(ctypes.cast(lv, ctypes.c_void_p), len(pack.dims), xcs, omcs, fptr(wp),
                                            Cout, N, C, Cout, stream())
            _t1(tok)
            ctx.save_for_backward(x, om, w)
        elif ctx.fused:
            wp = pack_weight2(w, dtype)[0]
            for l, (H, W) in enumerate(pack.dims):
                tok = _t0("adr::dcn_fwd_kernel(adr::DcnArgs)", *_dcn_work(N, H, W, C, Cout),
                          f"dcn fwd n{N} {H}x{W} c{C}->{Cout}" if _TIMING is not None else "", _reps())
                for _ in range(_reps()):
                    lib.adr_dcn_fwd_bf16(pack.at(xp, xcs, es, l), xcs, pack.at(omp, omcs, es, l), omcs, fptr(wp),
                                         pack.at(y.data_ptr(), Cout, es, l), Cout, N, H, W, C, Cout, stream())
                _t1(tok)
            ctx.save_for_backward(x, om, w)
        else:
            cols = torch.empty(pack.rows * 9 * C, dtype=dtype, device=dev)
            for l, (H, W) in enumerate(pack.dims):
                lib.adr_dcn_im2col(dcode(dtype), pack.at(xp, xcs, es, l), xcs, pack.at(omp, omcs, es, l), omcs,
                                   pack.at(cols.data_ptr(), 9 * C, es, l), N, H, W, C, stream())
            wp = pack_weight(w, dtype)
            d, _, _ = conv_desc(1, 1, pack.rows, 9 * C, 9 * C, Cout, 1, 1, 1, 1, 0, 0, Cout, dtype)
            conv_fwd(d, cols.data_ptr(), wp.data_ptr(), None, y.data_ptr())
            ctx.save_for_backward(x, om, cols, w)
        ctx.pw, ctx.pack = w, pack
        return y

    @staticmethod
    def backward(ctx, dy):
        pack = ctx.pack
        cols = None
        if ctx.fused:
            x, om, w = ctx.saved_tensors
        else:
            x, om, cols, w = ctx.saved_tensors
        dtype = x.dtype
        _, xp, xcs = nhwc(x)
        _, omp, omcs = nhwc(om)
        dy, dyp, dycs = nhwc(dy.to(dtype) if dy.dtype != dtype else dy)
        Np, C, _, S = x.shape
        Cout, omc = w.shape[0], om.shape[1]
        dev = x.device
        es = x.element_size()
        N = pack.N
        wt = torch.empty(9 * C * Cout, dtype=dtype, device=dev)
        lib.adr_dcn_weight_t(dcode(dtype), fptr(w.detach().float().contiguous()), fptr(wt), Cout, C, stream())
        dw = None
        if ctx.fused and not ctx.fused_bwd:
            cols = torch.empty(pack.rows * 9 * C, dtype=dtype, device=dev)
            for l, (H, W) in enumerate(pack.dims):
                lib.adr_dcn_im2col(dcode(dtype), pack.at(xp, xcs, es, l), xcs, pack.at(omp, omcs, es, l), omcs,
                                   pack.at(cols.data_ptr(), 9 * C, es, l), N, H, W, C, stream())
        if ctx.fused_bwd and DCN_LEVELS and len(pack.dims) <= 3:
            dx = pack.empty(C, dtype, dev)
            dom = pack.empty(omc, dtype, dev)
            lv = (DcnLevelStruct * len(pack.dims))()
            far = _dcn_far_scratch_levels(dev, N, pack.dims, C)
            for l, (H, W) in enumerate(pack.dims):
                lv[l].x, lv[l].om = pack.at(xp, xcs, es, l), pack.at(omp, omcs, es, l)
                lv[l].dy = pack.at(dyp, dycs, es, l)
                lv[l].dx, lv[l].dom = pack.at(dx.data_ptr(), C, es, l), pack.at(dom.data_ptr(), omc, es, l)
                lv[l].dxf, lv[l].flags = far[l][0].data_ptr(), far[l][1].data_ptr()
                lv[l].H, lv[l].W = H, W
            works = [_dcn_work(N, H, W, C, Cout) for H, W in pack.dims]
            nb = sum(w_[0] + 2 * N * H * W * C for w_, (H, W) in zip(works, pack.dims))
            tok = _t0("adr::dcn_bwd_levels_kernel(adr::DcnLevels)", nb, 2 * sum(w_[1] for w_ in works),
                      f"dcn bwd levels n{N} {pack.dims} c{C}->{Cout}" if _TIMING is not None else "")
            lib.adr_dcn_bwd_bf16_levels(ctypes.cast(lv, ctypes.c_void_p), len(pack.dims), xcs, omcs, dycs, fptr(wt),
                                        C, omc, N, C, Cout, stream())
            _t1(tok)
            if ctx.needs_input_grad[2]:
                stride = Cout * 9 * C
                splits = [lib.adr_dcn_wgrad_bf16_splits(N, H, W, C, Cout) for H, W in pack.dims]
                ws = torch.empty(sum(splits) * stride, dtype=torch.float32, device=dev)
                s0 = 0
                for l in range(len(pack.dims)):
                    lv[l].part, lv[l].splits = ws.data_ptr() + 4 * s0 * stride, splits[l]
                    s0 += splits[l]
                tok = _t0("adr::dcn_wgrad_levels_kernel(adr::DcnLevels)",
                          sum(w_[0] for w_ in works) + 4 * s0 * stride, sum(w_[1] for w_ in works),
                          f"dcn wgrad levels/{s0} n{N} {pack.dims} c{C}->{Cout}" if _TIMING is not None else "")
                lib.adr_dcn_wgrad_bf16_levels(ctypes.cast(lv, ctypes.c_void_p), len(pack.dims), xcs, omcs, dycs, N, C,
                                              Cout, stream())
                _t1(tok)
                out, ptr, acc = grad_dst(ctx.pw, stride, dev)
                if _dfr() is not None and acc and _TIMING is None:
                    _dfr().add(ws, stride, s0, ptr, Cout, C, C, 9, 0, acc)
                else:
                    lib.adr_wgrad_reduce_unpack(fptr(ws), stride, s0, ptr, Cout, C, C, 9, 0, acc, stream())
                dw = grad_ret(ctx.pw, out)
        elif ctx.fused_bwd:
            dx = pack.empty(C, dtype, dev)
            dom = pack.empty(omc, dtype, dev)
            for l, (H, W) in enumerate(pack.dims):
                dxf, flags = _dcn_far_scratch(dev, N, H, W, C)
                nb, fl = _dcn_work(N, H, W, C, Cout)
                tok = _t0("adr::dcn_bwd_kernel(adr::DcnArgs)", nb + 2 * N * H * W * C, 2 * fl,
                          f"dcn bwd n{N} {H}x{W} c{C}->{Cout}" if _TIMING is not None else "")
                lib.adr_dcn_bwd_bf16(pack.at(xp, xcs, es, l), xcs, pack.at(omp, omcs, es, l), omcs,
                                     pack.at(dyp, dycs, es, l), dycs, fptr(wt), pack.at(dx.data_ptr(), C, es, l), C,
                                     pack.at(dom.data_ptr(), omc, es, l), omc, fptr(dxf), fptr(flags), N, H, W, C,
                                     Cout, stream())
                _t1(tok)
            if ctx.needs_input_grad[2]:
                stride = Cout * 9 * C
                splits = [lib.adr_dcn_wgrad_bf16_splits(N, H, W, C, Cout) for H, W in pack.dims]
                ws = torch.empty(sum(splits) * stride, dtype=torch.float32, device=dev)
                s0 = 0
                for l, (H, W) in enumerate(pack.dims):
                    nb, fl = _dcn_work(N, H, W, C, Cout)
                    tok = _t0("adr::dcn_wgrad_kernel(adr::DcnArgs)", nb + 4 * splits[l] * stride, fl,
                              f"dcn wgrad/{splits[l]} n{N} {H}x{W} c{C}->{Cout}" if _TIMING is not None else "")
                    lib.adr_dcn_wgrad_bf16(pack.at(xp, xcs, es, l), xcs, pack.at(omp, omcs, es, l), omcs,
                                           pack.at(dyp, dycs, es, l), dycs,
                                           ctypes.c_void_p(ws.data_ptr() + 4 * s0 * stride), splits[l], N, H, W, C,
                                           Cout, stream())
                    _t1(tok)
                    s0 += splits[l]
                out, ptr, acc = grad_dst(ctx.pw, stride, dev)
                if _dfr() is not None and acc and _TIMING is None:
                    _dfr().add(ws, stride, s0, ptr, Cout, C, C, 9, 0, acc)
                else:
                    lib.adr_wgrad_reduce_unpack(fptr(ws), stride, s0, ptr, Cout, C, C, 9, 0, acc, stream())
                dw = grad_ret(ctx.pw, out)
        else:
            dx32 = zero_(torch.empty(pack.rows * C, dtype=torch.float32, device=dev))
            dom = zero_(pack.empty(omc, dtype, dev))
            dcols = torch.empty(pack.rows * 9 * C, dtype=dtype, device=dev)
            d, _, _ = conv_desc(1, 1, pack.rows, Cout, dycs, 9 * C, 1, 1, 1, 1, 0, 0, 9 * C, dtype)
            conv_fwd(d, dyp, wt.data_ptr(), None, dcols.data_ptr())
            if ctx.needs_input_grad[2]:
                dwd, _, _ = conv_desc(1, 1, pack.rows, 9 * C, 9 * C, Cout, 1, 1, 1, 1, 0, 0, dycs, dtype)
                dw = wgrad_param(ctx.pw, dwd, cols.data_ptr(), dyp, Cout, 9 * C, 1, w.shape, 0, dev)
            for l, (H, W) in enumerate(pack.dims):
                lib.adr_dcn_col2im(dcode(dtype), pack.at(xp, xcs, es, l), xcs, pack.at(omp, omcs, es, l), omcs,
                                   pack.at(dcols.data_ptr(), 9 * C, es, l), pack.at(dx32.data_ptr(), C, 4, l),
                                   pack.at(dom.data_ptr(), omc, es, l), omc, N, H, W, C, int(dtype == torch.float32),
                                   stream())
            dx = pack.empty(C, dtype, dev)
            lib.adr_cast(F32, fptr(dx32), dcode(dtype), ctypes.c_void_p(dx.data_ptr()), pack.rows * C, stream())
        return dx, dom, dw, None


def dcn_levels(x, om, w, pack):
    return LevelDCNFn.apply(x, om, w, pack)


class LevelAxisMeanFn(torch.autograd.Function):
    """CoordAtt's row / column means (AxisMeanFn 'coord', head.py:684-690) of every level of a packed activation, as
    ONE packed tensor of the pooled planes: `pp` = LevelPack(N, [(1, H_l + W_l)]), so an image's plane is its
    [H_l row means ; W_l column means] rows, and the 1x1 convs / BatchNorm after it run once for all levels."""

    @staticmethod
    def forward(ctx, x, pack, pp):
        vx = _v(x)
        C = x.shape[1]
        es = x.element_size()
        out = pp.empty(C, x.dtype, x.device)
        for l, (H, W) in enumerate(pack.dims):
            o = pp.at(out.data_ptr(), C, es, l).value
            lib.adr_axis_mean(dcode(x.dtype), pack.at(vx[1], vx[2], es, l), vx[2], pack.N, H, W, C,
                              ctypes.c_void_p(o), (H + W) * C, ctypes.c_void_p(o + H * C * es), (H + W) * C, stream())
        ctx.pack, ctx.pp, ctx.meta = pack, pp, (C, x.dtype)
        ctx.sink = _sink_of(x)
        return out

    @staticmethod
    def backward(ctx, dy):
        pack, pp = ctx.pack, ctx.pp
        C, dtype = ctx.meta
        _, dp, dcs = nhwc(dy)
        dx, acc = _dx_dst(ctx, (pack.Np, C, 1, pack.S), dtype, dy.device)
        es, xcs = dx.element_size(), dx.stride(3)
        for l, (H, W) in enumerate(pack.dims):
            o = pp.at(dp, dcs, es, l).value
            lib.adr_axis_mean_bwd(dcode(dtype), ctypes.c_void_p(o), (H + W) * dcs, ctypes.c_void_p(o + H * dcs * es),
                                  (H + W) * dcs, pack.at(dx.data_ptr(), xcs, es, l), xcs, pack.N, H, W, C, acc,
                                  stream())
        return (None if ctx.sink is not None else dx), None, None


def axis_mean_levels(x, pack, pp):
    return LevelAxisMeanFn.apply(x, pack, pp)


class LevelGateFn(torch.autograd.Function):
    """CoordAtt's output x * a_h * a_w (GateFn 'coord', head.py:704-706) per level of a packed activation; a_h / a_w
    are packed pooled planes (LevelAxisMeanFn's layout: the gate reads a_h's row-mean rows and a_w's column-mean
    rows of each image)."""

    @staticmethod
    def forward(ctx, x, ah, aw, pack, pp):
        ah, ahp, ahcs = nhwc(ah)
        aw, awp, awcs = nhwc(aw)
        vx = _v(x)
        C = x.shape[1]
        if ahcs != C or awcs != C:
            raise RuntimeError("gate_levels: a_h / a_w must be dense planes")
        es = x.element_size()
        out = pack.empty(C, x.dtype, x.device)
        for l, (H, W) in enumerate(pack.dims):
            lib.adr_gate(dcode(x.dtype), pack.at(vx[1], vx[2], es, l), vx[2], pp.at(ahp, C, es, l), (H + W) * C,
                         ctypes.c_void_p(pp.at(awp, C, es, l).value + H * C * es), (H + W) * C,
                         pack.at(out.data_ptr(), C, es, l), C, pack.N, H, W, C, stream())
        ctx.save_for_backward(vx[0], ah, aw)
        ctx.pack, ctx.pp = pack, pp
        ctx.sink = _sink_of(x)
        return out

    @staticmethod
    def backward(ctx, dout):
        pack, pp = ctx.pack, ctx.pp
        x, ah, aw = ctx.saved_tensors
        vx, vd = _v(x), _v(dout)
        C = x.shape[1]
        es = x.element_size()
        dx, acc = _dx_dst(ctx, (pack.Np, C, 1, pack.S), x.dtype, x.device)
        xcs = dx.stride(3)
        dah = pp.empty(C, x.dtype, x.device)
        daw = pp.empty(C, x.dtype, x.device)
        for l, (H, W) in enumerate(pack.dims):
            # zero_other: each gradient plane's unused rows (dah's column rows, daw's row rows) are written as 0
            _gate_bwd(dcode(x.dtype), pack.at(vx[1], vx[2], es, l).value, vx[2], pp.at(ah.data_ptr(), C, es, l).value,
                      (H + W) * C, pp.at(aw.data_ptr(), C, es, l).value + H * C * es, (H + W) * C,
                      pack.at(vd[1], vd[2], es, l).value, vd[2], pack.at(dx.data_ptr(), xcs, es, l).value, xcs,
                      pp.at(dah.data_ptr(), C, es, l).value, (H + W) * C,
                      pp.at(daw.data_ptr(), C, es, l).value + H * C * es, (H + W) * C, pack.N, H, W, C, acc, 1,
                      x.device)
        return (None if ctx.sink is not None else dx), dah, daw, None, None


def gate_levels(x, ah, aw, pack, pp):
    return LevelGateFn.apply(x, ah, aw, pack, pp)


class BNPackFn(torch.autograd.Function):
    """act(BatchNorm2d(y)) in training mode with per-LEVEL batch statistics over a packed activation (CoordAtt's bn1
    on the three levels' pooled planes, head.py:694-700): the reference calls the shared module once per level, so
    each level normalises with its own statistics and the running statistics are updated level by level."""

    @staticmethod
    def forward(ctx, y, pack, gamma, beta, rm, rv, act, momentum, eps):
        dtype = y.dtype
        y, yp, ycs = nhwc(y)
        Np, C, _, S = y.shape
        dev = y.device
        rows = _stats_rows(Np, S)
        chunks = lib.adr_nc_reduce_chunks(S, rows)
        part = torch.empty(Np * chunks * 2 * C, dtype=torch.float32, device=dev)
        scale = torch.empty(Np * C, dtype=torch.float32, device=dev)
        shift = torch.empty(Np * C, dtype=torch.float32, device=dev)
        mean = torch.empty(pack.L * C, dtype=torch.float32, device=dev)
        rstd = torch.empty(pack.L * C, dtype=torch.float32, device=dev)
        lib.adr_nc_reduce(dcode(dtype), 0, ctypes.c_void_p(yp), ycs, 0, None, 0, 0, None, None, 0, 0, Np, S, C, rows,
                          fptr(part), stream())
        lib.adr_bn_finalize_packed(fptr(part), pack.L, ctypes.cast(pack.k_c, ctypes.c_void_p), pack.N, chunks, S, C,
                                   fptr(gamma.detach()), fptr(beta.detach()), fptr(rm), fptr(rv), float(momentum),
                                   float(eps), fptr(scale), fptr(shift), fptr(mean), fptr(rstd), stream())
        z = pack.empty(C, dtype, dev)
        lib.adr_affine_act(dcode(dtype), ctypes.c_void_p(yp), ycs, 0, ctypes.c_void_p(z.data_ptr()), C, 0,
                           fptr(scale), fptr(shift), 1, ACT[act], Np, S, C, stream())
        ctx.save_for_backward(y, scale, shift, mean, rstd, gamma)
        ctx.meta = (act, chunks, rows)
        ctx.pack, ctx.pbeta = pack, beta
        return z

    @staticmethod
    def backward(ctx, dz):
        y, scale, shift, mean, rstd, gamma = ctx.saved_tensors
        act, chunks, rows = ctx.meta
        pack = ctx.pack
        dz, dzp, dzcs = nhwc(dz.to(y.dtype) if dz.dtype != y.dtype else dz)
        _, yp, ycs = nhwc(y)
        Np, C, _, S = y.shape
        dev = y.device
        dt = dcode(y.dtype)
        part = torch.empty(Np * chunks * 2 * C, dtype=torch.float32, device=dev)
        lib.adr_nc_reduce(dt, 1, ctypes.c_void_p(yp), ycs, 0, ctypes.c_void_p(dzp), dzcs, 0, fptr(scale),
                          fptr(shift), 1, ACT[act], Np, S, C, rows, fptr(part), stream())
        f = lambda: torch.empty(Np * C, dtype=torch.float32, device=dev)  # noqa: E731
        A, B, Cc = f(), f(), f()
        dgamma, pg, acc_g = grad_dst(gamma, C, dev)
        dbeta, pb, acc_b = grad_dst(ctx.pbeta, C, dev)
        if acc_g != acc_b:
            raise RuntimeError("BN gamma/beta gradients must share one destination kind")
        lib.adr_bn_bwd_finalize_packed(fptr(part), pack.L, ctypes.cast(pack.k_c, ctypes.c_void_p), pack.N, chunks, S,
                                       C, fptr(mean), fptr(rstd), fptr(gamma.detach()), pg, pb, fptr(A), fptr(B),
                                       fptr(Cc), acc_g, stream())
        dy = pack.empty(C, y.dtype, dev)
        lib.adr_affine_act_bwd(dt, ctypes.c_void_p(yp), ycs, 0, ctypes.c_void_p(dzp), dzcs, 0,
                               ctypes.c_void_p(dy.data_ptr()), C, 0, fptr(scale), fptr(shift), fptr(A), fptr(B),
                               fptr(Cc), 1, 1, ACT[act], Np, S, C, 0, stream())
        return dy, None, grad_ret(gamma, dgamma), grad_ret(ctx.pbeta, dbeta), None, None, None, None, None


def bn_act_packed(y, pack, bn, act):
    """Training BatchNorm + activation with per-level statistics over a packed activation (BNPackFn)."""
    return BNPackFn.apply(y, pack, bn.weight, bn.bias, bn.running_mean, bn.running_var, act, bn.momentum, bn.eps)


class ScaleLevelsFn(torch.autograd.Function):
    """x * s_l on level l of a packed activation (AYHead's per-level Scale modules, head.py:1176), written into
    `box` when given; the scalars' gradients are per-level dot sums (batched at the WGRAD flush)."""

    @staticmethod
    def forward(ctx, x, pack, box, *gs):
        vx = _v(x)
        Np, C, _, S = x.shape
        es = x.element_size()
        out, op, ocs = _out_view(box, Np, C, 1, S, x.dtype, x.device)
        gf = [g.detach().float().contiguous() for g in gs]
        for l, (H, W) in enumerate(pack.dims):
            lib.adr_bcast_mul(dcode(x.dtype), pack.at(vx[1], vx[2], es, l), vx[2], fptr(gf[l]), 0, 0, None, 0,
                              pack.at(op, ocs, es, l), ocs, pack.N, H * W, C, 0, stream())
        ctx.save_for_backward(vx[0], *gf)
        ctx.pack, ctx.params = pack, gs
        return out if box is None else out[:, :]

    @staticmethod
    def backward(ctx, dy):
        saved = ctx.saved_tensors
        x, gf = saved[0], saved[1:]
        pack = ctx.pack
        vd = _v(dy)
        C = x.shape[1]
        es = x.element_size()
        dx = None
        if ctx.needs_input_grad[0]:
            dx = pack.empty(C, x.dtype, x.device)
            for l, (H, W) in enumerate(pack.dims):
                lib.adr_bcast_mul(dcode(x.dtype), pack.at(vd[1], vd[2], es, l), vd[2], fptr(gf[l]), 0, 0, None, 0,
                                  pack.at(dx.data_ptr(), C, es, l), C, pack.N, H * W, C, 0, stream())
        dgs = []
        for l, p in enumerate(ctx.params):
            if not ctx.needs_input_grad[3 + l]:
                dgs.append(None)
                continue
            xl, dl = pack.view(x, l), pack.view(vd[0], l)
            if _defer_dot(p, xl, dl):
                out = torch.empty(1, dtype=torch.float32, device=x.device)
                _dfr().add_dotsum(xl, dl, out)
                dgs.append(sink(p, out.view(p.shape)))
            else:
                dgs.append(sink(p, _reduce_dot(xl, dl, True, True).view(p.shape)))
        return (dx, None, None, *dgs)


def scale_levels(x, gs, pack, out=None):
    return ScaleLevelsFn.apply(x, pack, None if out is None else OutBox(out), *gs)
