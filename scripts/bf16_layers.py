"""Per-layer bf16 vs fp32 divergence of the whole network (train or eval mode), both on the GPU with the same
recipe weights and images. Prints relative L2 of each layer's output (and of each head output).
usage: python scripts/bf16_layers.py [--train] [--img 320] [--bs 2]"""
import argparse
import sys
from pathlib import Path

import torch

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT / "yolo-ad-refine_amd"), str(ROOT / "oracle"), str(ROOT / "tests")]
from recipe import synthetic_images  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--train", action="store_true")
ap.add_argument("--img", type=int, default=320)
ap.add_argument("--bs", type=int, default=2)
args = ap.parse_args()

from adrefine.nn.tasks import DetectionModel  # noqa: E402
from gpu_util import load_recipe_into  # noqa: E402

CFG = ROOT / "tests" / "configs" / "yolo11-701-YOLO-AD-Refine.yaml"
x = synthetic_images(args.bs, args.img, seed=0).cuda()
outs = {}
for dt in (torch.float32, torch.bfloat16):
    m = DetectionModel(str(CFG), compute_dtype=dt)
    load_recipe_into(m)
    m = m.cuda().train(args.train)
    rec = outs[dt] = {}

    def hook(mod, inp, out, i=None):
        rec[mod.i] = out

    for layer in m.model:
        layer.register_forward_hook(hook)
    # sub-module hooks inside the head
    head = m.model[-1]
    for name, sub in head.named_modules():
        if name and name.count(".") == 0:
            sub.register_forward_hook(lambda mod, inp, out, n=name: rec.setdefault("h." + n, []).append(out))
    with torch.no_grad() if not args.train else torch.enable_grad():
        m(x)
    torch.cuda.synchronize()


def rel(a, b):
    if isinstance(a, (list, tuple)):
        return [rel(u, v) for u, v in zip(a, b) if torch.is_tensor(u)]
    a, b = a.detach().double(), b.detach().double()
    return round(float((a - b).norm() / (b.norm() + 1e-30)), 5)


for k in outs[torch.float32]:
    if k not in outs[torch.bfloat16]:
        continue
    a, b = outs[torch.bfloat16][k], outs[torch.float32][k]
    if isinstance(a, list) and k.startswith("h."):
        print(k, [rel(u, v) for u, v in zip(a, b)])
    else:
        print(k, rel(a, b))
