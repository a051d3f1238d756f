"""Time the flash attention (adr_attn_fwd / adr_attn_bwd) at the C2PTSSA MHA shape: bs 64, 2 heads of 64,
1200 tokens (3 stacked 20x20 scales), bf16 (env B, H, L, D, R: l-scale 1280^2 is B 16, H 4, L 4800); HIP events; prints achieved TFLOP/s (4*B*H*L^2*d fwd, 2.5x bwd)."""
import os
import sys
from pathlib import Path

import torch

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "yolo-ad-refine_amd"))
from adrefine import kernels as K  # noqa: E402

B, H, L, D, R = (int(os.environ.get(k, v)) for k, v in (("B", 64), ("H", 2), ("L", 1200), ("D", 64), ("R", 20)))
E = H * D
qkv = (torch.randn(B, 3 * E, L, 1, device="cuda") * 0.5).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
qkv.requires_grad_(True)
go = torch.randn(B, E, L, 1, device="cuda").to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
for _ in range(3):
    o = K.attention(qkv, H)
    o.backward(go)
torch.cuda.synchronize()
e = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
tf = tb = 0.0
for _ in range(R):
    e[0].record()
    o = K.attention(qkv, H)
    e[1].record()
    o.backward(go)
    e[2].record()
    torch.cuda.synchronize()
    tf += e[0].elapsed_time(e[1])
    tb += e[1].elapsed_time(e[2])
fl = 4.0 * B * H * L * L * D
print(f"fwd {1e3 * tf / R:.1f} us ({fl / (tf / R * 1e-3) / 1e12:.0f} TF/s)  bwd {1e3 * tb / R:.1f} us "
      f"({2.5 * fl / (tb / R * 1e-3) / 1e12:.0f} TF/s)")
