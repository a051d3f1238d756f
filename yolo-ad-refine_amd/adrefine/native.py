"""ctypes binding of libadr_hip.so. Prototypes are parsed from include/adr.h so the Python view of the ABI
cannot drift from the header. Every call checks the status and raises RuntimeError(adr_last_error())."""
from __future__ import annotations

import ctypes
import os
import re
from pathlib import Path

_HERE = Path(__file__).resolve().parent
LIB_PATH = Path(os.environ.get("ADR_LIB", _HERE / "lib" / "libadr_hip.so"))  # ADR_LIB: A/B builds (dev)
HEADER = Path(os.environ["ADR_HEADER"]) if "ADR_HEADER" in os.environ else _HERE.parents[1] / "include" / "adr.h"
if not HEADER.exists():  # installed layout: header shipped next to the library
    HEADER = _HERE / "lib" / "adr.h"


class ConvDesc(ctypes.Structure):
    _fields_ = [(n, ctypes.c_int) for n in (
        "n", "h", "w", "c", "x_cstride", "x_coff", "k", "r", "s", "stride_h", "stride_w", "pad_h", "pad_w",
        "ho", "wo", "y_cstride", "y_coff", "dtype")]


_STRUCTS = {"adr_conv_desc": ConvDesc}


def _ctype(t: str):
    t = t.replace("const", "").strip()
    ptr = t.endswith("*")
    base = t.rstrip("*").strip()
    if ptr:
        if base in _STRUCTS:
            return ctypes.POINTER(_STRUCTS[base])
        if base == "char":
            return ctypes.c_char_p
        return ctypes.c_void_p
    return {"int": ctypes.c_int, "double": ctypes.c_double, "float": ctypes.c_float, "size_t": ctypes.c_size_t,
            "long": ctypes.c_long, "uint8_t": ctypes.c_uint8, "int64_t": ctypes.c_int64, "void": None}[base]


def parse_header(path=HEADER):
    src = path.read_text()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    protos = {}
    for m in re.finditer(r"^\s*((?:const\s+)?[a-z_0-9]+\s*\**)\s*(adr_[a-z0-9_]+)\s*\(([^)]*)\)\s*;", src, re.M):
        ret, name, args = m.group(1), m.group(2), m.group(3)
        argt = []
        for a in args.split(","):
            a = a.strip()
            if not a or a == "void":
                continue
            a = re.sub(r"\b[a-zA-Z_][a-zA-Z_0-9]*$", "", a).strip()  # drop parameter name
            argt.append(_ctype(a))
        protos[name] = (_ctype(ret), argt)
    return protos


class _Lib:
    def __init__(self):
        if not LIB_PATH.exists():
            raise RuntimeError(f"libadr_hip.so not built at {LIB_PATH}; run __graft_entry__.build() "
                               "(make -C yolo-ad-refine_amd)")
        self.lib = ctypes.CDLL(str(LIB_PATH), mode=ctypes.RTLD_GLOBAL)
        self.protos = parse_header()
        self.lib.adr_last_error.restype = ctypes.c_char_p
        for name, (ret, args) in self.protos.items():
            fn = getattr(self.lib, name)  # AttributeError == missing export
            fn.restype = ret
            fn.argtypes = args

    def __getattr__(self, name):
        fn = getattr(self.lib, name)
        ret = self.protos[name][0]
        if ret is ctypes.c_int and name not in _NONSTATUS:
            def call(*a):
                if OP_TRACE is not None:
                    return _traced(name, fn, a)
                if CALL_HOOK is not None:
                    return CALL_HOOK(name, fn, a)
                rc = fn(*a)
                if rc != 0:
                    raise RuntimeError(f"{name}: {self.lib.adr_last_error().decode()}")
                return rc
            setattr(self, name, call)
            return call
        setattr(self, name, fn)
        return fn


# Measurement hook (kernels.timing_begin for bench.py's roofline): when set, status-returning entry points are
# called as CALL_HOOK(name, fn, args) -> status.
CALL_HOOK = None

# Development op tracer (scripts/op_table.py): when OP_TRACE is a list, every status-returning entry point is
# bracketed by HIP events on the current stream and recorded as (name, caller, int args, event0, event1).
OP_TRACE = None


def _traced(name, fn, a):
    import sys

    import torch
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    rc = fn(*a)
    e1.record()
    if rc != 0:
        raise RuntimeError(f"{name}: {lib.lib.adr_last_error().decode()}")
    caller = f"{sys._getframe(2).f_code.co_name}<{sys._getframe(3).f_code.co_name}"
    ints = []
    for v in a:  # integer arguments, and a conv descriptor's geometry (passed by reference)
        if isinstance(v, int) and not isinstance(v, bool) and abs(v) < (1 << 31):
            ints.append(v)
        elif isinstance(getattr(v, "_obj", None), ConvDesc):
            d = v._obj
            ints += [d.n, d.h, d.w, d.c, d.x_cstride, d.k, d.r, d.s, d.stride_h]
    ints = tuple(ints)
    OP_TRACE.append((name, caller, ints, e0, e1))
    return rc


_NONSTATUS = {"adr_abi_version", "adr_conv2d_wgrad_bias_fusable", "adr_dwconv_wgrad_bias_fusable", "adr_conv2d_fwd_stat_tiles", "adr_conv2d_fwd_bf16_stat_tiles", "adr_conv2d_wgrad_splits", "adr_nc_reduce_chunks", "adr_opt_entry_size", "adr_pack_chunk_size", "adr_pack_tile_size", "adr_stem_fwd_tiles",
              "adr_opt_chunk_size", "adr_dcn_wgrad_bf16_splits", "adr_gn_fused_supported",
              "adr_fp8_amax_blocks", "adr_conv2d_fp8_supported", "adr_conv2d_fwd_fp8_stat_tiles",
              "adr_dwconv_fwd_act_supported", "adr_conv2d_bf16_xf_reuse", "adr_augment_desc_size",
              "adr_dcn_bwd_tiles", "adr_conv2d_fwd_bf16_bnact_stat_tiles",
              "adr_conv2d_dgrad_bf16_stat_tiles", "adr_conv2d_wgrad_batched_tile"}
_ = _NONSTATUS

lib = _Lib()
assert lib.lib.adr_abi_version() == 1, "ABI version mismatch"
