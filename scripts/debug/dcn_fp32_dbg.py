"""Locate the fp32 parity-path doffset error at C=256 (tests/test_gpu_dcn.py case6)."""
import sys
from pathlib import Path
ROOT = Path(__file__).resolve().parents[2]
sys.path[:0] = [str(ROOT / "tests"), str(ROOT / "oracle"), str(ROOT / "yolo-ad-refine_amd")]
import torch
from test_gpu_dcn import _inputs, _oracle, _run
for case in [(1, 256, 256, 40, 40, 4.0), (1, 192, 192, 40, 40, 4.0), (1, 128, 128, 40, 40, 4.0), (1, 256, 256, 16, 16, 4.0)]:
    N, C, Cout, H, W, spread = case
    x, om, w, gy = _inputs(N, C, Cout, H, W, spread, seed=7)
    ry, rdx, rdom, rdw = _oracle(x, om, w, gy)
    y, dx, dom, dw = _run(x, om, w, gy, torch.float32)
    e = (dom[:, :27] - rdom[:, :27]).abs()
    m = float(rdom[:, :18].abs().max())
    bad = (e > 1e-3 * m).nonzero()
    print(case, "max err/max", float(e[:, :18].max()) / m, "n bad", len(bad), "first", bad[:8].tolist())
    if len(bad):
        n, ch, h, ww = bad[0].tolist()
        print("  got", float(dom[n, ch, h, ww]), "want", float(rdom[n, ch, h, ww]), "om", om[n, :18, h, ww].tolist())
