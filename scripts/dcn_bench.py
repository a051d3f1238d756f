"""Time the DCN forward / backward at the AYHead shapes (bs 64, 64 -> 64 channels, 80/40/20 maps, bf16) with HIP
events; ADR_DCN_FUSED=0 selects the im2col + GEMM + col2im path for an A/B. Env N, C, SIZES (e.g. N=16 C=256
SIZES=160,80,40 for the l-scale head at 1280), SPREAD (offset range in px)."""
import os
import sys
from pathlib import Path

import torch

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "yolo-ad-refine_amd"))
from adrefine import kernels as K  # noqa: E402

torch.manual_seed(0)
tot_f = tot_b = 0.0
SPREAD = float(os.environ.get("SPREAD", "1"))
for S in [int(v) for v in os.environ.get("SIZES", "80,40,20").split(",")]:
    N, C = int(os.environ.get("N", 64)), int(os.environ.get("C", 64))
    x = torch.randn(N, C, S, S, device="cuda").to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    om = torch.zeros(N, 32, S, S, device="cuda")
    om[:, :18] = (torch.rand(N, 18, S, S, device="cuda") * 2 - 1) * SPREAD
    om[:, 18:27] = torch.randn(N, 9, S, S, device="cuda")
    om = om.to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    w = (torch.randn(C, C, 3, 3, device="cuda") * 0.05).requires_grad_(True)
    xg, omg = x.clone().requires_grad_(True), om.clone().requires_grad_(True)
    gy = torch.randn(N, C, S, S, device="cuda").to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    for _ in range(3):
        y = K.dcn(xg, omg, w)
        y.backward(gy)
    torch.cuda.synchronize()
    e = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
    tf = tb = 0.0
    R = 10
    for _ in range(R):
        e[0].record()
        y = K.dcn(xg, omg, w)
        e[1].record()
        y.backward(gy)
        e[2].record()
        torch.cuda.synchronize()
        tf += e[0].elapsed_time(e[1])
        tb += e[1].elapsed_time(e[2])
    tot_f += tf / R
    tot_b += tb / R
    print(f"{S}x{S}: fwd {1e3 * tf / R:.1f} us  bwd {1e3 * tb / R:.1f} us", flush=True)
print(f"total fwd {1e3 * tot_f:.1f} us  bwd {1e3 * tot_b:.1f} us  sum {1e3 * (tot_f + tot_b):.1f} us")
