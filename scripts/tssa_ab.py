"""TSSA kernels of the in-tree library against another build (default ab/tssa_old.so, the 256-thread kernels) on
the same inputs: forward (out, Pi, ss, attn) and backward (dq, dk, dv, dtemp), fp32 and bf16; the in-tree kernel
is also run twice with garbage pre-filled outputs (determinism / uninitialised reads).
usage: python scripts/tssa_ab.py [other.so]   (GPU)"""
import ctypes, sys
from pathlib import Path
ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "yolo-ad-refine_amd"))
import torch
import adrefine.kernels as K
from adrefine.native import lib

other = ctypes.CDLL(str(ROOT / (sys.argv[1] if len(sys.argv) > 1 else "ab/tssa_old.so")))
vp = ctypes.c_void_p
for L in (lib, other):
    L.adr_tssa_fwd.argtypes = [ctypes.c_int, vp, vp, vp, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                               ctypes.c_int, vp, vp, ctypes.c_int, ctypes.c_int, vp, vp, vp, vp]
    L.adr_tssa_bwd.argtypes = [ctypes.c_int, vp, vp, vp, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                               ctypes.c_int, vp, vp, ctypes.c_int, ctypes.c_int, vp, vp, vp, vp, vp, vp, ctypes.c_int,
                               vp, vp, vp]


def run(L, dt, B, N, heads, fill):
    torch.manual_seed(0)
    D = 64
    C = heads * D
    qkv = torch.randn(B, N, 3 * C, device="cuda").to(dt)
    temp = torch.rand(heads, device="cuda") + 0.5
    dout = torch.randn(B, N, C, device="cuda").to(dt)
    out = torch.full((B, N, C), fill, device="cuda").to(dt)
    Pi = torch.full((B, heads, N), fill, device="cuda"); ss = torch.full_like(Pi, fill)
    att = torch.full((B, heads, D), fill, device="cuda")
    g = torch.full((B, N, 3 * C), fill, device="cuda").to(dt)
    dtemp = torch.full((heads,), fill, device="cuda"); ws = torch.full((B * heads,), fill, device="cuda")
    code = 1 if dt == torch.float32 else 2
    es = qkv.element_size(); p = qkv.data_ptr()
    P = lambda t: vp(t.data_ptr())
    assert L.adr_tssa_fwd(K.dcode(dt), vp(p), vp(p + C * es), vp(p + 2 * C * es), 3 * C, B, N, heads, D, P(temp),
                          P(out), C, N, P(Pi), P(ss), P(att), vp(K.stream())) == 0
    gp = g.data_ptr()
    assert L.adr_tssa_bwd(K.dcode(dt), vp(p), vp(p + C * es), vp(p + 2 * C * es), 3 * C, B, N, heads, D, P(temp),
                          P(dout), C, N, P(Pi), P(ss), P(att), vp(gp), vp(gp + C * es), vp(gp + 2 * C * es), 3 * C,
                          P(dtemp), P(ws), vp(K.stream())) == 0
    torch.cuda.synchronize()
    return dict(out=out.float(), Pi=Pi, ss=ss, att=att, dq=g[..., :C].float(), dk=g[..., C:2 * C].float(),
                dv=g[..., 2 * C:].float(), dtemp=dtemp)


for dt in (torch.float32, torch.bfloat16):
    for B, N, heads in ((4, 100, 2), (4, 400, 4), (2, 1600, 4)):
        a, a2, b = run(lib, dt, B, N, heads, 7.0), run(lib, dt, B, N, heads, -3.0), run(other, dt, B, N, heads, 7.0)
        msg = []
        for k in a:
            rel = float((a[k] - b[k]).abs().max() / b[k].abs().max().clamp_min(1e-30))
            msg.append(f"{k} {rel:.1e}{'' if torch.equal(a[k], a2[k]) else ' NONDET'}")
        print(str(dt)[6:], B, N, heads, " | ".join(msg), flush=True)
