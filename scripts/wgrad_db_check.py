"""Digest of the bf16 WGRAD partials + reduce over a set of 128 x 128-tile shapes (fixed seeds), for comparing two
kernel selections bitwise across processes, e.g. ADR_WG_DB=0 vs 1:
usage: ADR_WG_DB=0 python scripts/wgrad_db_check.py; ADR_WG_DB=1 python scripts/wgrad_db_check.py   (GPU)"""
import ctypes, hashlib, sys
from pathlib import Path
ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "yolo-ad-refine_amd"))
import torch
import adrefine.kernels as K
from adrefine.native import lib

SHAPES = [(4, 40, 40, 128, 128, 1, 1, 1), (2, 20, 20, 256, 128, 3, 3, 2), (3, 17, 13, 192, 160, 3, 3, 1),
          (1, 9, 7, 136, 200, 1, 1, 1), (8, 80, 80, 128, 256, 1, 1, 1), (2, 31, 33, 256, 256, 3, 3, 2)]
h = hashlib.sha256()
for i, (N, H, W, C, Kc, R, S, st) in enumerate(SHAPES):
    g = torch.Generator(device="cuda").manual_seed(100 + i)
    d, Ho, Wo = K.conv_desc(N, H, W, C, C, Kc, R, S, st, st, R // 2, S // 2, Kc, torch.bfloat16)
    x = torch.randn(N * H * W * C, device="cuda", generator=g).to(torch.bfloat16)
    dy = torch.randn(N * Ho * Wo * Kc, device="cuda", generator=g).to(torch.bfloat16)
    splits = lib.adr_conv2d_wgrad_splits(ctypes.byref(d))
    ws = torch.empty(splits * Kc * R * S * C, device="cuda")
    dw = torch.empty(Kc * R * S * C, device="cuda")
    lib.adr_conv2d_wgrad_partials(ctypes.byref(d), K.fptr(x), K.fptr(dy), K.fptr(ws), 0, K.stream())
    lib.adr_wgrad_reduce(K.fptr(ws), K.fptr(dw), dw.numel(), splits, 0, K.stream())
    ref = torch.einsum("pk,pc->kc", dy.float().view(-1, Kc), x.float().view(-1, C)) if (R, st) == (1, 1) else None
    torch.cuda.synchronize()
    if ref is not None:
        err = float((dw.view(Kc, C) - ref).abs().max() / ref.abs().max())
        assert err < 1e-5, (SHAPES[i], err)
    h.update(dw.cpu().numpy().tobytes())
    print(SHAPES[i], "splits", splits, hashlib.sha256(dw.cpu().numpy().tobytes()).hexdigest()[:16])
print("digest", h.hexdigest())
