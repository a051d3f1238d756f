"""CPU-side checks of the C-ABI library: it loads, and exports every symbol include/adr.h declares."""
import ctypes
import re

from conftest import ROOT

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
