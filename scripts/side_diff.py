"""Which parameter gradients change when the side stream is on: one fp32 forward+backward through the trainer with
ADR_SIDE_STREAM on and off, arena slices compared per parameter. usage: python scripts/side_diff.py (GPU)"""
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "yolo-ad-refine_amd"))
sys.path.insert(0, str(ROOT / "tests"))
sys.path.insert(0, str(ROOT / "oracle"))
import torch

import adrefine.kernels as K
from adrefine.engine.trainer import FusedTrainer
from adrefine.nn.tasks import DetectionModel
from gpu_util import load_recipe_into
from recipe import synthetic_images, synthetic_labels

CFG = ROOT / "tests/configs/yolo11-701-YOLO-AD-Refine.yaml"
res = {}
for on in (False, True, True):
    K._SIDE_ON = on
    m = DetectionModel(str(CFG))
    load_recipe_into(m)
    m = m.cuda()
    tr = FusedTrainer(m, lr0=0.01, momentum=0.937, weight_decay=5e-4, nbs=2, batch_size=2)
    x = synthetic_images(2, 320, seed=0)
    lab = synthetic_labels(2, 80, seed=1)
    b = tr._prepare({"img": x.cuda(), **lab})
    tr.forward_backward(b)
    torch.cuda.synchronize()
    g = {n: tr.param_grad(n).clone() for n, t, _, isp in tr.entries if isp}
    res.setdefault(on, []).append(g)
base = res[False][0]
for run in res[True]:
    diffs = []
    for n, v in base.items():
        w = run[n]
        d = float((v - w).norm() / (v.norm() + 1e-12))
        if d > 1e-6:
            diffs.append((d, n))
    diffs.sort(reverse=True)
    print(len(diffs), "params differ; worst:", diffs[:12], flush=True)
