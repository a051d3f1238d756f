"""Stem (model.0 Conv(3, K, 3, 2) on the uint8 batch) forward / weight-gradient timing through the C ABI at the
step's shape (bs 64, 640^2, K 16), with the algorithmic bytes (image read once, y / dy once) per launch.
usage: python scripts/stem_micro.py [N] [S] [K] [reps]   (GPU)"""
import ctypes, sys
from pathlib import Path
ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "yolo-ad-refine_amd"))
import torch
import adrefine.kernels as K
from adrefine.native import lib

N = int(sys.argv[1]) if len(sys.argv) > 1 else 64
S = int(sys.argv[2]) if len(sys.argv) > 2 else 640
Kc = int(sys.argv[3]) if len(sys.argv) > 3 else 16
reps = int(sys.argv[4]) if len(sys.argv) > 4 else 20
Ho = (S - 1) // 2 + 1
torch.manual_seed(0)
img = torch.randint(0, 256, (N, 3, S, S), dtype=torch.uint8, device="cuda")
w = torch.randn(Kc, 3, 3, 3, device="cuda") * 0.1
y = torch.empty(N * Ho * Ho * Kc, dtype=torch.bfloat16, device="cuda")
stats = torch.empty(lib.adr_stem_fwd_tiles(N, Ho) * 2 * Kc, device="cuda")
dy = torch.randn(N * Ho * Ho * Kc, device="cuda").to(torch.bfloat16)
dw = torch.empty(Kc * 27, device="cuda")
wsb = lib.adr_stem_wgrad_workspace(N, S, S, Kc)
ws = torch.empty(wsb // 4 + 1, device="cuda")
s = K.stream()


def fwd():
    assert lib.adr_stem_conv_fwd_u8(K.fptr(img), N, S, S, K.fptr(w), Kc, ctypes.c_void_p(y.data_ptr()), Kc,
                                    K.fptr(stats), s) == 0


def wgrad():
    assert lib.adr_stem_conv_wgrad_u8(K.fptr(img), N, S, S, ctypes.c_void_p(dy.data_ptr()), Kc, Kc, K.fptr(dw), 0,
                                      K.fptr(ws), wsb, s) == 0


def timed(f):
    for _ in range(3):
        f()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize(); e0.record()
    for _ in range(reps):
        f()
    e1.record(); torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e-3


import os
nb_img, nb_y = img.numel(), y.numel() * 2
outs = {}
for var in ("0", "1"):  # the previous kernels (env 0) against the current ones
    os.environ["ADR_STEM_FWD_Q"] = var
    os.environ["ADR_STEM_WG_Q"] = var
    for name, f, nb in (("fwd", fwd, nb_img + nb_y), ("wgrad", wgrad, nb_img + nb_y)):
        t = timed(f)
        print(f"[{var}] stem {name} N{N} {S}^2 K{Kc}: {t * 1e6:7.1f} us  {nb / t / 1e12:5.2f} TB/s algorithmic "
              f"({nb / 1e6:.0f} MB)", flush=True)
    fwd(); wgrad(); torch.cuda.synchronize()
    outs[var] = (y.float().clone(), stats.clone(), dw.clone())
for name, a, b in zip(("y", "stats", "dw"), outs["0"], outs["1"]):
    rel = float((a - b).abs().max() / b.abs().max().clamp_min(1e-30))
    print(f"{name}: max|new-old|/max|old| = {rel:.3e}  bitwise {torch.equal(a, b)}")
