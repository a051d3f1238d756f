"""Probe of the BiFPN fusion-weight gradient (model.28): the per-input dot sum(x_i * dy), |x_i * dy| and |dy|
seen by FusionFn.backward, for the fp32 and bf16 HIP paths (the fp32 reference: 21.86 / 3497 / 8145, -24.30 /
3459 / 8145)."""
import sys
sys.path.insert(0, "tests"); sys.path.insert(0, "yolo-ad-refine_amd"); sys.path.insert(0, "oracle")
import torch
from conftest import golden
import test_gpu_grads as T
from adrefine import kernels as K

rec = []
orig = K.FusionFn.backward


def bwd(ctx, dy):
    fwd, w, *xs = ctx.saved_tensors
    d = dy.double()
    rec.append([(float((x.double() * d).sum()), float((x.double() * d).abs().sum()), float(d.abs().sum()),
                 float(x.double().abs().sum())) for x in xs])
    return orig(ctx, dy)


K.FusionFn.backward = staticmethod(bwd)
g = golden("net701_grads_320")
for dt in (torch.float32, torch.bfloat16):
    rec.clear()
    _, mine = T._hip_grads(dt, g)
    print(dt, [[tuple(round(v, 3) for v in r) for r in e] for e in rec], mine["model.28.fusion_weight"].tolist())
