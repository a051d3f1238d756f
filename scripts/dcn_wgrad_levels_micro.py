"""Time adr_dcn_wgrad_bf16_levels (the AYHead's three DCN levels in one launch) and the three per-level
adr_dcn_wgrad_bf16 launches with HIP events. Env: N, C (= Cout), S (P3 map side; P4 = S/2, P5 = S/4), R (repeats)."""
import ctypes
import os
import sys
from pathlib import Path
ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "yolo-ad-refine_amd"))
import torch  # noqa: E402
import adrefine.kernels as K  # noqa: E402
from adrefine.native import lib  # noqa: E402
N, C, S, R = (int(os.environ.get(k, d)) for k, d in (("N", 64), ("C", 64), ("S", 80), ("R", 10)))
dev = "cuda"
dims = [(S, S), (S // 2, S // 2), (S // 4, S // 4)]
lv = (K.DcnLevelStruct * 3)()
keep, splits = [], []
for l, (H, W) in enumerate(dims):
    x = torch.randn(N, H, W, C, device=dev).to(torch.bfloat16)
    om = torch.zeros(N, H, W, 32, device=dev)
    om[..., :18] = torch.rand(N, H, W, 18, device=dev) * 2 - 1
    om = om.to(torch.bfloat16)
    dy = torch.randn(N, H, W, C, device=dev).to(torch.bfloat16)
    sp = lib.adr_dcn_wgrad_bf16_splits(N, H, W, C, C)
    part = torch.empty(sp * 9 * C * C, dtype=torch.float32, device=dev)
    lv[l].x, lv[l].om, lv[l].dy, lv[l].part, lv[l].H, lv[l].W, lv[l].splits = (
        x.data_ptr(), om.data_ptr(), dy.data_ptr(), part.data_ptr(), H, W, sp)
    keep += [x, om, dy, part]
    splits.append(sp)


def levels():
    lib.adr_dcn_wgrad_bf16_levels(ctypes.cast(lv, ctypes.c_void_p), 3, C, 32, C, N, C, C, K.stream())


def per_level():
    for l in range(3):
        lib.adr_dcn_wgrad_bf16(ctypes.c_void_p(lv[l].x), C, ctypes.c_void_p(lv[l].om), 32, ctypes.c_void_p(lv[l].dy),
                               C, ctypes.c_void_p(lv[l].part), lv[l].splits, N, lv[l].H, lv[l].W, C, C, K.stream())


for name, fn in (("levels", levels), ("per-level", per_level)):
    for _ in range(2):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(R):
        fn()
    e1.record()
    torch.cuda.synchronize()
    print(f"dcn wgrad {name} N{N} C{C} P3 {S}x{S} splits {splits}: {e0.elapsed_time(e1) / R * 1000:.1f} us", flush=True)
