"""Time adr_dcn_bwd_bf16 alone (HIP events) at one AYHead shape. Env: N, C, S (map side), SPREAD (offset px),
ADR_DCN_BWD_MODE (1 / 2: skip the dom / dx phase, A/B only)."""
import os
import sys
from pathlib import Path
ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "yolo-ad-refine_amd"))
import ctypes  # noqa: E402
import torch  # noqa: E402
import adrefine.kernels as K  # noqa: E402
from adrefine.native import lib  # noqa: E402
N, C, S = int(os.environ.get("N", 64)), int(os.environ.get("C", 64)), int(os.environ.get("S", 80))
spread = float(os.environ.get("SPREAD", "1"))
dev = "cuda"
x = torch.randn(N, S, S, C, device=dev).to(torch.bfloat16)
om = torch.zeros(N, S, S, 32, device=dev)
om[..., :18] = (torch.rand(N, S, S, 18, device=dev) * 2 - 1) * spread
om[..., 18:27] = torch.randn(N, S, S, 9, device=dev)
om = om.to(torch.bfloat16)
dy = torch.randn(N, S, S, C, device=dev).to(torch.bfloat16)
wt = (torch.randn(9 * C * C, device=dev) * 0.05).to(torch.bfloat16)
dx = torch.empty_like(x)
dom = torch.empty_like(om)
dxf, flags = K._dcn_far_scratch(dev, N, S, S, C)
def run():
    lib.adr_dcn_bwd_bf16(K.fptr(x), C, K.fptr(om), 32, K.fptr(dy), C, K.fptr(wt), K.fptr(dx), C, K.fptr(dom), 32,
                         K.fptr(dxf), K.fptr(flags), N, S, S, C, C, K.stream())
for _ in range(3):
    run()
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
R = int(os.environ.get("R", 20))
e0.record()
for _ in range(R):
    run()
e1.record()
torch.cuda.synchronize()
print(f"dcn_bwd N{N} C{C} {S}x{S} spread {spread} mode {os.environ.get('ADR_DCN_BWD_MODE', '0')}: "
      f"{e0.elapsed_time(e1) / R * 1000:.1f} us/launch pair", flush=True)
