"""Check the bf16 conv kernels against fp32 PyTorch on the same bf16-rounded operands: forward output, input
gradient and weight gradient, relative L2 and max error (the kernel accumulates in fp32 and rounds the output
once to bf16, so errors sit at bf16 rounding level ~2^-9 relative)."""
import sys
from pathlib import Path

import torch
import torch.nn.functional as F

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "yolo-ad-refine_amd"))
from adrefine import kernels as K  # noqa: E402

torch.manual_seed(0)
worst = 0.0
for (n, c, k, r, s, hw) in [(8, 64, 64, 1, 1, 40), (8, 128, 128, 1, 1, 20), (8, 48, 64, 1, 1, 40), (4, 64, 128, 3, 2, 40),
                            (4, 128, 128, 3, 2, 40), (4, 16, 32, 3, 2, 64), (4, 64, 64, 3, 1, 40), (4, 256, 128, 1, 1, 20),
                            (4, 32, 256, 1, 1, 20)]:
    x = torch.randn(n, c, hw, hw, device="cuda").to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    w = (torch.randn(k, c, r, r, device="cuda") / (c * r * r) ** 0.5).to(torch.bfloat16).float()
    x.requires_grad_(True)
    wp = w.clone().requires_grad_(True)
    y, st = K.conv2d(x, wp, None, s, r // 2, True)
    gy = torch.randn(y.shape, device="cuda").to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    y.backward(gy)
    xr = x.detach().float().requires_grad_(True)
    wr = w.clone().requires_grad_(True)
    yr = F.conv2d(xr, wr, None, s, r // 2)
    yr.backward(gy.float())
    def rel(a, b):
        return float((a.float() - b).norm() / b.norm())
    e = (rel(y, yr), rel(x.grad, xr.grad), rel(wp.grad, wr.grad))
    # BN partial stats: sum over all tiles must equal the per-channel sum / sumsq of the stored bf16 output
    yf = y.detach().float()
    tot = st.view(-1, 2, k).sum(0)
    es = float((tot[0] - yf.sum((0, 2, 3))).abs().max() / yf.abs().sum((0, 2, 3)).max())
    worst = max(worst, *e, es)
    print(f"n{n} c{c} k{k} {r}x{r} s{s} hw{hw}: y {e[0]:.2e}  dx {e[1]:.2e}  dw {e[2]:.2e}  stats {es:.2e}", flush=True)
print(f"worst {worst:.2e}")
