"""Seeded, reference-free recipes for parity inputs — TEST INFRASTRUCTURE ONLY.

The same recipe is used (a) by oracle/gen_golden.py to load weights into the imported reference and
(b) by tests / smoke / bench to load the identical weights into the HIP build and the CPU oracle, so golden
fixtures never need to carry the 4.1 M parameters themselves.

Weights (one generator per state_dict key, seed 1000 + key index, keys in reference order):
  * running_mean -> 0.1 N;  running_var -> 1 + 0.1 |N|;  num_batches_tracked -> 0
  * dfl.conv.weight -> arange(16) (frozen in the reference, block.py:63-81)
  * named scalars/vectors (SPECIAL below) -> default + 0.1 N
  * tensors with >= 2 dims -> N * fan_in^-1/2 (fan_in = prod(shape[1:]))
  * '...bias' -> 0.1 N;  other 1-D 'weight' (BN / GN / LN / DyT affine) -> 1 + 0.1 N
Images: torch.rand(B, 3, S, S) with generator seed `seed` (default 0).
Labels ("COCO-shape"): per image n ~ Poisson(7.3) clipped [1, 93]; cls ~ U{0..nc-1};
centres ~ U(0.05, 0.95); w, h = exp(U(ln 0.02, ln 0.6)) clipped to the image; packed as the reference's
collate_fn (data/dataset.py:230-246): batch_idx (N,), cls (N, 1), bboxes (N, 4) normalised xywh.
"""
from __future__ import annotations

import math

import torch

SPECIAL = {
    "fusion_weight": 1.0, "fft": 1.0, "scale": 1.0, "scale_weights": 1.0 / 3, "stage_attention": 1.0 / 3,
    "residual_weight1": 0.1, "residual_weight2": 0.1, "temps": 1.0, "temp": 1.0, "alpha": 0.5,
    "gamma": 1e-6, "gammax": 1.0,
}


def recipe_tensor(idx: int, key: str, shape, dtype=torch.float32) -> torch.Tensor:
    g = torch.Generator().manual_seed(1000 + idx)
    leaf = key.rsplit(".", 1)[-1]
    shape = tuple(shape)
    if leaf == "num_batches_tracked":
        return torch.zeros(shape, dtype=torch.int64)
    n = torch.randn(shape, generator=g, dtype=torch.float32)
    if leaf == "running_mean":
        t = 0.1 * n
    elif leaf == "running_var":
        t = 1 + 0.1 * n.abs()
    elif key.endswith("dfl.conv.weight"):
        t = torch.arange(shape[1], dtype=torch.float32).view(shape)
    elif leaf == "alphas":
        t = torch.linspace(0.3, 1.0, shape[1]).view(shape) + 0.1 * n
    elif leaf in SPECIAL:
        t = SPECIAL[leaf] + 0.1 * n
    elif len(shape) >= 2:
        fan_in = max(1, math.prod(shape[1:]))
        t = n * fan_in ** -0.5
    elif "bias" in leaf:
        t = 0.1 * n
    else:
        t = 1 + 0.1 * n
    return t.to(dtype)


def recipe_state_dict(keys_shapes) -> dict:
    """keys_shapes: ordered iterable of (key, shape[, dtype]). Returns an ordered dict of tensors."""
    out = {}
    for idx, item in enumerate(keys_shapes):
        key, shape = item[0], item[1]
        out[key] = recipe_tensor(idx, key, shape)
    return out


def seeded_randn(*shape, seed: int = 11) -> torch.Tensor:
    """Module-fixture inputs: torch.randn(shape) from a fresh generator seeded `seed`."""
    return torch.randn(*shape, generator=torch.Generator().manual_seed(seed))


def synthetic_images(bs: int, size: int, seed: int = 0) -> torch.Tensor:
    g = torch.Generator().manual_seed(seed)
    return torch.rand(bs, 3, size, size, generator=g)


def synthetic_labels(bs: int, nc: int = 80, seed: int = 1, mean_n: float = 7.3, max_n: int = 93):
    g = torch.Generator().manual_seed(seed)
    rates = torch.full((bs,), mean_n)
    counts = torch.poisson(rates, generator=g).clamp(1, max_n).long()
    bi, cl, bx = [], [], []
    for j in range(bs):
        n = int(counts[j])
        c = torch.randint(0, nc, (n,), generator=g)
        ctr = 0.05 + 0.9 * torch.rand(n, 2, generator=g)
        lo, hi = math.log(0.02), math.log(0.6)
        wh = torch.exp(lo + (hi - lo) * torch.rand(n, 2, generator=g))
        wh = torch.minimum(wh, 2 * torch.minimum(ctr, 1 - ctr))  # keep the box inside the image
        bi.append(torch.full((n,), float(j)))
        cl.append(c.float().view(-1, 1))
        bx.append(torch.cat((ctr, wh), 1))
    return {"batch_idx": torch.cat(bi), "cls": torch.cat(cl), "bboxes": torch.cat(bx)}


def synthetic_predictions(bs: int, na: int, nc: int = 80, img: int = 640, seed: int = 7):
    """Eval-head-shaped predictions (bs, 4+nc, na) for NMS parity: xywh boxes in pixels + class scores.

    Built from torch.rand / randperm with exactly-rounded arithmetic only (no exp/log/sigmoid/randn, whose CPU
    vector code paths differ in the last ulp between ISAs), so any host regenerates identical bits and the
    NMS comparison can be bit-exact. Half the anchors are jittered copies of 64 "object" boxes per image, so
    suppression is real; scores are distinct within an image (a permutation raised to the 16th power), so the
    reference's unstable argsort cannot reorder ties. conf 0.25 keeps almost every anchor (single-label),
    conf 0.001 keeps about a third of all (anchor, class) pairs and exercises the max_nms cut."""
    g = torch.Generator().manual_seed(seed)
    xy = torch.rand(bs, 2, na, generator=g) * img
    u = torch.rand(bs, 2, na, generator=g)
    wh = 4 + 296 * (u * u * u)
    nobj = 64
    obj_xy = torch.rand(bs, 2, nobj, generator=g) * img
    ov = torch.rand(bs, 2, nobj, generator=g)
    obj_wh = 16 + 200 * (ov * ov)
    pick = torch.randint(0, nobj, (bs, na), generator=g)
    jit = torch.rand(bs, 4, na, generator=g)
    clustered = torch.rand(bs, na, generator=g) < 0.5
    cxy = torch.gather(obj_xy, 2, pick[:, None].expand(bs, 2, na)) + (jit[:, :2] - 0.5) * 8
    cwh = torch.gather(obj_wh, 2, pick[:, None].expand(bs, 2, na)) * (0.9 + 0.2 * jit[:, 2:])
    xy = torch.where(clustered[:, None], cxy, xy)
    wh = torch.where(clustered[:, None], cwh, wh)
    n = nc * na
    r = torch.stack([(torch.randperm(n, generator=g).to(torch.float32) + 0.5) / n for _ in range(bs)])
    s = r * r
    s = s * s
    s = s * s
    s = s * s
    return torch.cat((xy, wh, s.view(bs, nc, na)), 1)


AUG_SHAPES = [(1.0, 0.75), (0.625, 1.0), (1.0, 1.0), (0.78, 1.0), (1.0, 0.5625), (1.0, 0.906), (0.5, 1.0),
              (0.875, 0.875)]


def synthetic_aug_items(n: int, imgsz: int, seed: int = 3):
    """Training-augmentation inputs (data/augment.py fixtures): n BGR uint8 HWC images already resized as
    BaseDataset.load_image leaves them (long side = imgsz, data/base.py:151-172) with smooth gradients + noise,
    and per-image labels (cls (k, 1) float32, normalised xywh boxes (k, 4) float32, 1 <= k <= 8)."""
    g = torch.Generator().manual_seed(seed)
    items = []
    for i in range(n):
        fh, fw = AUG_SHAPES[i % len(AUG_SHAPES)]
        h, w = max(8, int(round(imgsz * fh))), max(8, int(round(imgsz * fw)))
        yy = torch.arange(h, dtype=torch.float32).view(h, 1, 1)
        xx = torch.arange(w, dtype=torch.float32).view(1, w, 1)
        ph = torch.rand(1, 1, 3, generator=g) * 6.0
        base = 127.5 + 80 * torch.sin(xx * 0.05 + yy * 0.031 + ph) + 30 * torch.cos(yy * 0.09 - ph)
        img = (base + torch.rand(h, w, 3, generator=g) * 40 - 20).clamp(0, 255).round().to(torch.uint8).numpy()
        k = int(torch.randint(1, 9, (1,), generator=g))
        ctr = 0.1 + 0.8 * torch.rand(k, 2, generator=g)
        wh = 0.05 + 0.45 * torch.rand(k, 2, generator=g)
        wh = torch.minimum(wh, 2 * torch.minimum(ctr, 1 - ctr))
        cls = torch.randint(0, 80, (k, 1), generator=g).float()
        items.append({"img": img, "cls": cls.numpy(), "bboxes": torch.cat((ctr, wh), 1).numpy()})
    return items


AUG_HYPS = {  # default.yaml training augmentation values (cfg/default.yaml) and a rotated / sheared / v-flipped set
    "default": dict(mosaic=1.0, degrees=0.0, translate=0.1, scale=0.5, shear=0.0, perspective=0.0, flipud=0.0,
                    fliplr=0.5, hsv_h=0.015, hsv_s=0.7, hsv_v=0.4, mixup=0.0, copy_paste=0.0,
                    copy_paste_mode="flip", bgr=0.0),
    "rot": dict(mosaic=1.0, degrees=10.0, translate=0.2, scale=0.6, shear=3.0, perspective=0.0, flipud=0.5,
                fliplr=0.5, hsv_h=0.03, hsv_s=0.8, hsv_v=0.5, mixup=0.0, copy_paste=0.0, copy_paste_mode="flip",
                bgr=0.0),
}
