"""A/B of the streaming 1x1 conv kernel (conv1_kernel) against the per-tile kernel at the step's 1x1 shapes, bf16,
with BatchNorm statistics: time per launch (HIP events, 20 reps) and HBM rate on the algorithmic bytes
(x + y once + w). Run once with ADR_CONV1=1 and once with ADR_CONV1=0 (the dispatch reads it at first use)."""
import ctypes
import os
import sys
from pathlib import Path
ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "yolo-ad-refine_amd"))
import torch  # noqa: E402
import adrefine.kernels as K  # noqa: E402
from adrefine.native import lib  # noqa: E402

SHAPES = [(64, 160, 160, 32, 32), (64, 80, 80, 64, 64), (64, 80, 80, 128, 64), (64, 40, 40, 128, 128),
          (64, 160, 160, 48, 32), (64, 80, 80, 96, 64), (64, 20, 20, 256, 128), (64, 80, 80, 64, 128),
          (16, 160, 160, 256, 128), (16, 80, 80, 256, 256), (16, 160, 160, 192, 64), (64, 40, 40, 256, 64)]
dt = torch.bfloat16
s = K.stream()
tag = os.environ.get("ADR_CONV1", "1")
for N, H, W, C, Kc in SHAPES:
    for mode in ("fwd", "dgrad"):
        if mode == "fwd":
            d, _, _ = K.conv_desc(N, H, W, C, C, Kc, 1, 1, 1, 1, 0, 0, Kc, dt)
            src = torch.randn(N * H * W * C, device="cuda").to(dt)
            out = torch.empty(N * H * W * Kc, device="cuda", dtype=dt)
            w = torch.randn(Kc * C, device="cuda").to(dt)
            tiles = lib.adr_conv2d_fwd_bf16_stat_tiles(ctypes.byref(d))
            st = torch.empty(tiles * 2 * Kc, device="cuda")
            run = lambda: lib.adr_conv2d_fwd_bf16(ctypes.byref(d), K.fptr(src), K.fptr(w), None, K.fptr(out),  # noqa
                                                  K.fptr(st), 0, s)
        else:
            d, _, _ = K.conv_desc(N, H, W, C, C, Kc, 1, 1, 1, 1, 0, 0, Kc, dt)
            src = torch.randn(N * H * W * Kc, device="cuda").to(dt)
            out = torch.empty(N * H * W * C, device="cuda", dtype=dt)
            w = torch.randn(Kc * C, device="cuda").to(dt)
            run = lambda: lib.adr_conv2d_dgrad_bf16(ctypes.byref(d), K.fptr(src), K.fptr(w), None, K.fptr(out), 0, s)  # noqa
        for _ in range(3):
            run()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(20):
            run()
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) / 20 * 1000
        nbytes = 2 * (N * H * W * (C + Kc) + C * Kc)
        print(f"conv1={tag} {mode:5s} n{N} {H}x{W} {C}->{Kc}: {us:7.1f} us  {nbytes / us / 1e3:6.0f} GB/s "
              f"({nbytes / us / 1e3 / 8000:.2f} of peak)", flush=True)
