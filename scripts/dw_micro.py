"""Time the depthwise conv kernels (forward, data gradient, weight gradient) at the C2PTSSA / EDFFN shapes
(bs 64, 20x20; 128 channels with k = 3 and 7, 512 channels with k = 3), bf16, HIP events."""
import sys
from pathlib import Path

import torch

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "yolo-ad-refine_amd"))
from adrefine import kernels as K  # noqa: E402

R = 20
tot = 0.0
for C, k in ((128, 3), (128, 7), (512, 3)):
    x = torch.randn(64, C, 20, 20, device="cuda").to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    x.requires_grad_(True)
    w = (torch.randn(C, 1, k, k, device="cuda") * 0.1).requires_grad_(True)
    b = torch.zeros(C, device="cuda", requires_grad=True)
    gy = torch.randn_like(x)
    for _ in range(3):
        y = K.dwconv(x, w, b, k)
        y.backward(gy)
    torch.cuda.synchronize()
    e = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
    tf = tb = 0.0
    for _ in range(R):
        e[0].record()
        y = K.dwconv(x, w, b, k)
        e[1].record()
        y.backward(gy)
        e[2].record()
        torch.cuda.synchronize()
        tf += e[0].elapsed_time(e[1])
        tb += e[1].elapsed_time(e[2])
    tot += (tf + tb) / R
    print(f"C{C} k{k}: fwd {1e3 * tf / R:.1f} us  bwd {1e3 * tb / R:.1f} us", flush=True)
print(f"total {1e3 * tot:.1f} us")
