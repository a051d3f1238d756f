"""CPU-side checks of the C-ABI library: it loads, and exports every symbol include/adr.h declares."""
import ctypes
import re

from conftest import PKG_ROOT, ROOT

LIB = ROOT / "yolo-ad-refine_amd" / "adrefine" / "lib" / "libadr_hip.so"
HDR = ROOT / "include" / "adr.h"


def _declared():
    src = re.sub(r"/\*.*?\*/", "", HDR.read_text(), flags=re.S)
    return re.findall(r"^\s*(?:const\s+)?[a-z_0-9]+\s*\**\s*(adr_[a-z0-9_]+)\s*\(", src, re.M)


def test_library_exports_all_declared_symbols():
    lib = ctypes.CDLL(str(LIB))
    names = _declared()
    assert len(names) >= 10
    missing = [n for n in names if not hasattr(lib, n)]
    assert not missing, missing
    lib.adr_abi_version.restype = ctypes.c_int
    assert lib.adr_abi_version() == 1


def test_python_binding_parses_header():
    import adrefine.native as N
    assert set(N.parse_header()) == set(_declared())


def test_one_hip_runtime_loaded():
    """Importing the package first (bench.py imports engine/ddp.py before anything else) must not load a second HIP
    runtime: libadr_hip.so binds to torch's libamdhip64, not /opt/rocm's (two runtimes in one process broke graph
    replay and the NMS occupancy query in round 6)."""
    import subprocess
    import sys
    code = ("import sys; sys.path.insert(0, %r); import adrefine.engine.ddp; "
            "m = open('/proc/self/maps').read(); "
            "print(sorted({l.split()[-1] for l in m.splitlines() if 'libamdhip64' in l}))") % str(PKG_ROOT)
    out = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=300).stdout.strip()
    libs = eval(out)  # noqa: S307 - our own printed list
    assert len(libs) == 1 and "torch" in libs[0], libs


def test_roofline_byte_estimators_take_ctypes_pointers():
    """bench.py's roofline timing hands every entry point's arguments, ctypes pointers included, to the per-entry
    byte / flop estimators (kernels._BATCHED_BYTES, _ALG_FLOPS); they must read c_void_p arguments (CPU check)."""
    import ctypes
    from adrefine import kernels as K
    tab = ctypes.c_void_p(0x1234000)
    f = K._BATCHED_BYTES["adr_pack_weight2_tiled"]
    assert f((1, tab, 7, None)) == 0
    K._PACK_BYTES[0x1234000] = 4096
    try:
        assert f((1, tab, 7, None)) == 4096
    finally:
        del K._PACK_BYTES[0x1234000]
    p = ctypes.c_void_p(1)
    fwd = (1, p, p, p, 384, 0, 128, 256, 64, p, 128, 2, 100, 2, 64, 64, 0.125, p, None)
    assert K._ALG_FLOPS["adr_attn_fwd"](fwd) == 2.0 * 2 * 2 * 100 ** 2 * 128
    bwd = (1, p, p, p, 384, 0, 128, 256, 64, p, 128, p, 128, p, p, p, p, 384, 0, 128, 256, 2, 100, 2, 64, 64, 0.125,
           p, None)
    assert K._ALG_FLOPS["adr_attn_bwd"](bwd) == 2.0 * 2 * 2 * 100 ** 2 * (3 * 64 + 2 * 64)
