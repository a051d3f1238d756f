"""Forward conv kernel time, bf16 engine vs fp8 engine (incl. the per-call weight pack), at l-scale 1280^2 bs16
shapes. usage: python scripts/fp8_micro.py (GPU)"""
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "yolo-ad-refine_amd"))
import torch

from adrefine import kernels as K

SHAPES = [(64, 128, 320, 3, 1), (128, 128, 320, 3, 1), (128, 128, 320, 1, 1), (128, 256, 320, 3, 2),
          (256, 256, 160, 3, 1), (256, 256, 160, 1, 1), (256, 512, 160, 3, 2), (512, 512, 80, 3, 1),
          (512, 512, 80, 1, 1), (512, 512, 40, 3, 1), (1024, 512, 40, 1, 1)]


def bench(fn, reps=10):
    for _ in range(2):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / reps


for c1, c2, hw, k, s in SHAPES:
    x = torch.randn(16, c1, hw, hw, device="cuda").to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    w = torch.randn(c2, c1, k, k, device="cuda") * 0.02
    out = {}
    for fp8 in (False, True):
        K.CONV_FP8 = fp8
        out[fp8] = bench(lambda: K.conv2d(x, w, None, s, k // 2, want_stats=True))
    fl = 2 * 16 * (hw // s) ** 2 * c2 * c1 * k * k
    print(f"c{c1}->{c2} {hw}^2 k{k} s{s}: bf16 {out[False]:8.1f} us ({fl / out[False] / 1e6:6.0f} TF/s)  "
          f"fp8 {out[True]:8.1f} us ({fl / out[True] / 1e6:6.0f} TF/s)", flush=True)
    del x
