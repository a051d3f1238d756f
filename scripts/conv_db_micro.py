"""A/B of the double-buffered narrow conv tile (conv_bf16_db_kernel, ADR_CONV_DB) against the single-buffered one on
the generic implicit-GEMM shapes of the n-scale step (20^2 stride-1 3x3, stride-2 3x3 forward / data gradient):
bitwise check of the two outputs, then HIP-event times of each (ADR_CONV_DB is read per call).
usage: python scripts/conv_db_micro.py [reps]   (GPU)"""
import ctypes, os, sys
from pathlib import Path
ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "yolo-ad-refine_amd"))
import torch
import adrefine.kernels as K
from adrefine.native import lib

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 50
dt = torch.bfloat16
# (mode, N, H, W, C, K, R, S, stride)
SHAPES = [("fwd", 64, 20, 20, 64, 64, 3, 3, 1), ("fwd", 64, 20, 20, 128, 64, 3, 3, 1),
          ("fwd", 64, 20, 20, 32, 32, 3, 3, 1), ("fwd", 64, 20, 20, 16, 16, 3, 3, 1),
          ("fwd", 64, 40, 40, 64, 64, 3, 3, 2), ("fwd", 64, 80, 80, 64, 64, 3, 3, 2),
          ("fwd", 64, 160, 160, 32, 32, 3, 3, 2), ("fwd", 64, 40, 40, 32, 32, 3, 3, 2),
          ("dgrad", 64, 20, 20, 64, 64, 3, 3, 1), ("dgrad", 64, 20, 20, 32, 32, 3, 3, 1),
          ("dgrad", 64, 40, 40, 64, 64, 3, 3, 2), ("dgrad", 64, 40, 40, 16, 16, 3, 3, 2)]
s = K.stream()
for mode, N, H, W, C, Kc, R, S, st in SHAPES:
    d, Ho, Wo = K.conv_desc(N, H, W, C, C, Kc, R, S, st, st, R // 2, S // 2, Kc, dt)
    torch.manual_seed(0)
    x = torch.randn(N * H * W * C, device="cuda").to(dt)
    w4 = (torch.randn(Kc, R, S, C, device="cuda") * 0.05).to(dt)
    w = w4.reshape(-1).contiguous()
    wt = w4.permute(3, 1, 2, 0).contiguous().reshape(-1)
    y = torch.randn(N * Ho * Wo * Kc, device="cuda").to(dt)
    out = y if mode == "fwd" else x
    stats = torch.zeros(2 * Kc * 65536 if mode == "fwd" else 1, device="cuda")

    def run():
        if mode == "fwd":
            rc = lib.adr_conv2d_fwd_bf16(ctypes.byref(d), K.fptr(x), K.fptr(w), None, K.fptr(y), K.fptr(stats), 0, s)
        else:
            rc = lib.adr_conv2d_dgrad_bf16(ctypes.byref(d), K.fptr(y), K.fptr(wt), None, K.fptr(x), 0, s)
        assert rc == 0, rc

    res, times = [], []
    for v in ("0", "-1"):
        os.environ["ADR_CONV_DB"] = v
        out.zero_(); stats.zero_(); run(); torch.cuda.synchronize()
        res.append((out.clone(), stats.clone()))
        for _ in range(3):
            run()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize(); e0.record()
        for _ in range(reps):
            run()
        e1.record(); torch.cuda.synchronize()
        times.append(e0.elapsed_time(e1) / reps * 1e3)
    same = torch.equal(res[0][0], res[1][0]) and torch.equal(res[0][1], res[1][1])
    print(f"{mode:5s} N{N} {H}x{W} C{C} K{Kc} s{st}: single {times[0]:6.1f} us  db {times[1]:6.1f} us  "
          f"bitwise {'yes' if same else 'NO'}", flush=True)
