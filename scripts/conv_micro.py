"""Time one conv contraction (fwd / dgrad / wgrad) at a given shape through the C ABI; fwd2/dgrad2 run the bf16
engine (adr_conv.hip) and check it against the generic engine on the same inputs.
usage: python scripts/conv_micro.py MODE N H W C K R S STRIDE [reps]   (bf16, pad = R//2)"""
import ctypes, sys
from pathlib import Path
ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "yolo-ad-refine_amd"))
import torch
import adrefine.kernels as K
from adrefine.native import lib

mode = sys.argv[1]
N, H, W, C, Kc, R, S, st = (int(v) for v in sys.argv[2:10])
reps = int(sys.argv[10]) if len(sys.argv) > 10 else 20
dt = torch.bfloat16
d, Ho, Wo = K.conv_desc(N, H, W, C, C, Kc, R, S, st, st, R // 2, S // 2, Kc, dt)
x = torch.randn(N * H * W * C, device="cuda").to(dt)
w4 = torch.randn(Kc, R, S, C, device="cuda").to(dt)           # KRSC
w = w4.reshape(-1).contiguous()
wt = w4.permute(3, 1, 2, 0).contiguous().reshape(-1)         # CRSK
y = torch.randn(N * Ho * Wo * Kc, device="cuda").to(dt)
splits = lib.adr_conv2d_wgrad_splits(ctypes.byref(d))
ws = torch.empty(splits * Kc * R * S * C, device="cuda")
dw = torch.empty(Kc * R * S * C, device="cuda")
s = K.stream()

def run(m=mode):
    if m == "fwd":
        lib.adr_conv2d_fwd(ctypes.byref(d), K.fptr(x), K.fptr(w), None, K.fptr(y), None, 0, s)
    elif m == "fwd2":
        lib.adr_conv2d_fwd_bf16(ctypes.byref(d), K.fptr(x), K.fptr(w), None, K.fptr(y), None, 0, s)
    elif m == "dgrad":
        lib.adr_conv2d_dgrad(ctypes.byref(d), K.fptr(y), K.fptr(w), None, K.fptr(x), 0, s)
    elif m == "dgrad2":
        lib.adr_conv2d_dgrad_bf16(ctypes.byref(d), K.fptr(y), K.fptr(wt), None, K.fptr(x), 0, s)
    else:
        lib.adr_conv2d_wgrad_partials(ctypes.byref(d), K.fptr(x), K.fptr(y), K.fptr(ws), 0, s)
        lib.adr_wgrad_reduce(K.fptr(ws), K.fptr(dw), dw.numel(), splits, 0, s)

err = ""
if mode in ("fwd2", "dgrad2"):
    out = y if mode == "fwd2" else x
    run(mode[:-1]); torch.cuda.synchronize(); ref = out.float().clone()
    out.zero_(); run(mode); torch.cuda.synchronize()
    rel = float((out.float() - ref).abs().max() / ref.abs().max())
    err = f"  max|d|/max|ref|={rel:.2e}"
    if rel > 2e-2:
        print("MISMATCH", mode, sys.argv[2:10], err)
        sys.exit(1)
for _ in range(3):
    run()
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(reps):
    run()
e1.record()
torch.cuda.synchronize()
t = e0.elapsed_time(e1) / reps * 1e-3
nb, fl = K._conv_work(d)
print(f"{mode} {' '.join(sys.argv[2:10])}: {t * 1e6:.1f} us  {nb / t / 1e9:.0f} GB/s  {fl / t / 1e12:.1f} TF/s{err}")
