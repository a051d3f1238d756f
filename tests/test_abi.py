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
