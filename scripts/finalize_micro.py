"""Per-launch time of the BatchNorm finalize kernels (adr_bn_finalize / adr_bn_bwd_finalize) against the number of
partial rows P and channels C: 50 back-to-back launches captured in one hipGraph and replayed (the train step's
setting), so the figure is kernel time + the inter-kernel gap. usage: python scripts/finalize_micro.py (GPU)"""
import os
import sys
from pathlib import Path

import torch

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "yolo-ad-refine_amd"))
from adrefine import kernels as K  # noqa: E402
from adrefine.native import lib  # noqa: E402

fp = K.fptr
for C in (8, 16, 32, 64, 128, 256):
    for P in (400, 1600, 3200, 6400, 12800, 25600):
        part = torch.rand(P * 2 * C, device="cuda")
        g = torch.ones(C, device="cuda"); b = torch.zeros(C, device="cuda")
        rm = torch.zeros(C, device="cuda"); rv = torch.ones(C, device="cuda")
        sc, sh, mu, rs = (torch.empty(C, device="cuda") for _ in range(4))
        A, B, Cc, dg, db = (torch.empty(C, device="cuda") for _ in range(5))
        s = torch.cuda.Stream()
        res = []
        for kind, mode in (("fwd", "0"), ("fwd", "1"), ("bwd", "0"), ("bwd", "1")):
            os.environ["ADR_FIN_PRESUM"] = mode
            def run():
                st = K.stream()
                for _ in range(50):
                    if kind == "fwd":
                        lib.adr_bn_finalize(fp(part), P, C, float(P * 128), fp(g), fp(b), fp(rm), fp(rv), 0.03, 1e-3, 1,
                                            fp(sc), fp(sh), fp(mu), fp(rs), st)
                    else:
                        lib.adr_bn_bwd_finalize(fp(part), P, C, float(P * 128), fp(mu), fp(rs), fp(g), fp(dg), fp(db),
                                                fp(A), fp(B), fp(Cc), 1, 0, st)
            with torch.cuda.stream(s):
                run()
            torch.cuda.synchronize()
            gr = torch.cuda.CUDAGraph()
            with torch.cuda.graph(gr, stream=s):
                run()
            gr.replay(); torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(5):
                gr.replay()
            e1.record(); torch.cuda.synchronize()
            res.append(e0.elapsed_time(e1) * 1e3 / 250)
        print(f"C {C:4d} P {P:6d}: fwd {res[0]:6.2f} -> {res[1]:6.2f} us  bwd {res[2]:6.2f} -> {res[3]:6.2f} us "
              "(single launch -> pre-summed)")
