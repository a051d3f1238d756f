"""Time adr_dcn_col2im alone at the AYHead P3 shape (bs 64, 64 ch, 80x80)."""
import ctypes, os, sys
from pathlib import Path
ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "yolo-ad-refine_amd"))
import torch
import adrefine.kernels as K
from adrefine.native import lib
N, C, H, W = int(os.environ.get("N", 64)), 64, 80, 80
dev = "cuda"
g = torch.Generator(device="cpu").manual_seed(0)
x = torch.randn(N, H, W, C, generator=g).to(dev, torch.bfloat16)
om = torch.randn(N, H, W, 32, generator=g).to(dev, torch.bfloat16)
dcols = torch.randn(N * H * W * 9 * C, generator=g).to(dev, torch.bfloat16)
dx32 = torch.zeros(N * H * W * C, device=dev)
dom = torch.zeros(N, H, W, 32, device=dev, dtype=torch.bfloat16)
def run():
    lib.adr_dcn_col2im(1, K.fptr(x), C, K.fptr(om), 32, K.fptr(dcols), K.fptr(dx32), K.fptr(dom), 32, N, H, W, C, K.stream())
for _ in range(3): run()
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(10): run()
e1.record(); torch.cuda.synchronize()
print(f"variant {os.environ.get('ADR_DCN_VARIANT', '0')}: {e0.elapsed_time(e1) / 10 * 1000:.1f} us")
