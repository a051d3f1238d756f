"""adr_ew at the step's shapes (bf16): add (fan-out sum), mul, act; HIP events, 20 reps. ADR_EW_ROWS selects the
rows-per-thread instantiation (1 / 2 / 4)."""
import ctypes
import os
import sys
from pathlib import Path
ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "yolo-ad-refine_amd"))
import torch  # noqa: E402
import adrefine.kernels as K  # noqa: E402
from adrefine.native import lib  # noqa: E402
s = K.stream()
for N, H, W, C in [(64, 160, 160, 32), (64, 80, 80, 64), (64, 40, 40, 128), (64, 20, 20, 256), (64, 80, 80, 128)]:
    a = torch.randn(N * H * W * C, device="cuda").to(torch.bfloat16)
    b = torch.randn_like(a)
    o = torch.empty_like(a)
    for op, name, nb in ((1, "axpby", 3), (4, "act", 2)):
        run = lambda: lib.adr_ew(1, op, 1, K.fptr(a), C, K.fptr(b) if op == 1 else None, C, None, 0, K.fptr(o), C,  # noqa
                                 N * H * W, C, None, None, 0, s)
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
        by = nb * a.numel() * 2
        print(f"rows={os.environ.get('ADR_EW_ROWS', '4')} {name:5s} {N}x{H}x{W}x{C}: {us:6.1f} us {by / us / 1e3:6.0f} GB/s",
              flush=True)
