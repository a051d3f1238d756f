"""Time the BatchNorm streaming kernels (adr_affine_act, adr_affine_act_bwd, adr_nc_reduce stats / bwd) at the
701-n bs-64 activation shapes with HIP events; prints us and algorithmic GB/s per launch."""
import ctypes
import sys
from pathlib import Path

import torch

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "yolo-ad-refine_amd"))
from adrefine import kernels as K  # noqa: E402
from adrefine.native import lib  # noqa: E402

SHAPES = [(64, 320, 16), (64, 160, 32), (64, 160, 64), (64, 80, 64), (64, 80, 128), (64, 40, 128), (64, 20, 256)]
R = 20


FLUSH = torch.empty(512 << 20, dtype=torch.uint8, device="cuda")  # > the 256 MB Infinity Cache


def timed(fn):
    """Average of R launches, each preceded by an (untimed-in-effect) cache flush: per-launch event pairs."""
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    tot = 0.0
    for _ in range(R):
        FLUSH.zero_()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        torch.cuda.synchronize()
        tot += a.elapsed_time(b)
    return 1e3 * tot / R


tot = {}
for N, S, C in SHAPES:
    HW = S * S
    y = torch.randn(N * HW * C, device="cuda").to(torch.bfloat16)
    dz = torch.randn(N * HW * C, device="cuda").to(torch.bfloat16)
    z = torch.empty_like(y)
    dx = torch.empty_like(y)
    sc = torch.rand(C, device="cuda") + 0.5
    sh = torch.randn(C, device="cuda") * 0.1
    A, B, Cc = (torch.randn(C, device="cuda") * 0.1 for _ in range(3))
    rows = K._stats_rows(N, HW)
    chunks = lib.adr_nc_reduce_chunks(HW, rows)
    part = torch.empty(N * chunks * 2 * C, device="cuda")
    P = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
    st = K.stream()
    nb = y.numel() * 2
    res = {
        "affine_act": (timed(lambda: lib.adr_affine_act(1, P(y), C, 0, P(z), C, 0, K.fptr(sc), K.fptr(sh), 0, 1, N, HW,
                                                         C, st)), 2 * nb),
        "affine_act_bwd": (timed(lambda: lib.adr_affine_act_bwd(1, P(y), C, 0, P(dz), C, 0, P(dx), C, 0, K.fptr(sc),
                                                                 K.fptr(sh), K.fptr(A), K.fptr(B), K.fptr(Cc), 0, 0, 1,
                                                                 N, HW, C, 0, st)), 3 * nb),
        "nc_reduce_stats": (timed(lambda: lib.adr_nc_reduce(1, 0, P(y), C, 0, None, 0, 0, None, None, 0, 0, N, HW, C,
                                                             rows, K.fptr(part), st)), nb),
        "nc_reduce_bwd": (timed(lambda: lib.adr_nc_reduce(1, 1, P(y), C, 0, P(dz), C, 0, K.fptr(sc), K.fptr(sh), 0, 1,
                                                           N, HW, C, rows, K.fptr(part), st)), 2 * nb),
    }
    line = []
    for k, (us, by) in res.items():
        tot[k] = tot.get(k, 0.0) + us
        line.append(f"{k} {us:7.1f}us {by / us / 1e3:6.0f}GB/s")
    print(f"N{N} {S}x{S} C{C} ({nb / 1e6:.0f} MB): " + " | ".join(line), flush=True)
print("totals(us): " + ", ".join(f"{k} {v:.1f}" for k, v in tot.items()))

# adr_ew copy / axpby at the same shapes
tot = {}
for N, S, C in SHAPES:
    HW = S * S
    a = torch.randn(N * HW * C, device="cuda").to(torch.bfloat16)
    b = torch.randn_like(a)
    o = torch.empty_like(a)
    P = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
    st = K.stream()
    nb = a.numel() * 2
    res = {"ew_copy": (timed(lambda: lib.adr_ew(1, 0, 0, P(a), C, None, 0, None, 0, P(o), C, N * HW, C, None, None, 0,
                                                 st)), 2 * nb),
           "ew_axpby": (timed(lambda: lib.adr_ew(1, 1, 0, P(a), C, P(b), C, None, 0, P(o), C, N * HW, C, None, None, 0,
                                                  st)), 3 * nb)}
    line = []
    for k, (us, by) in res.items():
        tot[k] = tot.get(k, 0.0) + us
        line.append(f"{k} {us:7.1f}us {by / us / 1e3:6.0f}GB/s")
    print(f"N{N} {S}x{S} C{C}: " + " | ".join(line), flush=True)
print("totals(us): " + ", ".join(f"{k} {v:.1f}" for k, v in tot.items()))
