"""Synthetic COCO-shape training batches — the bench's input stream. No dataset is
available offline: images are torch.rand (already /255-normalised, as after detect/train.py:57-59) and labels
follow COCO's per-image statistics, packed like YOLODataset.collate_fn (data/dataset.py:230-246):
batch_idx (N,), cls (N, 1), bboxes (N, 4) normalised xywh. The test oracle generates the same stream from the
same recipe (tests/test_synthetic.py checks they agree)."""
from __future__ import annotations

import math

import torch


def images(bs: int, size: int, seed: int = 0) -> torch.Tensor:
    g = torch.Generator().manual_seed(seed)
    return torch.rand(bs, 3, size, size, generator=g)


def images_u8(bs: int, size: int, seed: int = 0) -> torch.Tensor:
    """The dataloader's form of a batch: uint8 NCHW (YOLODataset.collate_fn stacks uint8 images; the trainer's
    preprocess_batch divides by 255 on the device, detect/train.py:57-59)."""
    g = torch.Generator().manual_seed(seed)
    return torch.randint(0, 256, (bs, 3, size, size), generator=g, dtype=torch.uint8)


def labels(bs: int, nc: int = 80, seed: int = 1, mean_n: float = 7.3, max_n: int = 93):
    """Per image n ~ Poisson(mean_n) clipped to [1, max_n]; cls ~ U{0..nc-1}; centre ~ U(0.05, 0.95)^2;
    w, h = exp(U(ln 0.02, ln 0.6)) shrunk to stay inside the image."""
    g = torch.Generator().manual_seed(seed)
    counts = torch.poisson(torch.full((bs,), mean_n), generator=g).clamp(1, max_n).long()
    bi, cl, bx = [], [], []
    lo, hi = math.log(0.02), math.log(0.6)
    for j in range(bs):
        n = int(counts[j])
        c = torch.randint(0, nc, (n,), generator=g)
        ctr = 0.05 + 0.9 * torch.rand(n, 2, generator=g)
        wh = torch.exp(lo + (hi - lo) * torch.rand(n, 2, generator=g))
        wh = torch.minimum(wh, 2 * torch.minimum(ctr, 1 - ctr))
        bi.append(torch.full((n,), float(j)))
        cl.append(c.float().view(-1, 1))
        bx.append(torch.cat((ctr, wh), 1))
    return {"batch_idx": torch.cat(bi), "cls": torch.cat(cl), "bboxes": torch.cat(bx)}


def train_batch(bs: int, img: int, seed: int, device, nc: int = 80, u8: bool = False):
    """Device-resident batch for FusedTrainer.step: {'img': (bs,3,img,img) fp32 in [0, 1] (or the uint8 batch the
    dataloader yields, u8=True), 'gt': (bs, nmax, 5)}."""
    from ..utils.loss import preprocess_targets
    lab = labels(bs, nc, seed=seed + 1)
    gt = preprocess_targets(lab["batch_idx"], lab["cls"], lab["bboxes"], bs, (img, img)).to(device)
    im = images_u8(bs, img, seed=seed) if u8 else images(bs, img, seed=seed)
    return {"img": im.to(device), "gt": gt}, lab


def head_output(bs: int, na: int = 8400, nc: int = 80, img: int = 640, seed: int = 7, objects: int = 64):
    """A decoded eval-head output (bs, 4 + nc, na) fp32 with controlled NMS work, for the bench's NMS leg: xywh boxes
    in pixels, half of the anchors jittered copies of `objects` boxes per image (real suppression), class scores
    s = u^16 with u a per-image permutation of (k + 0.5) / (nc * na) — distinct within an image, and ~30 % of all
    (anchor, class) pairs above the validator's conf 0.001 (the max_nms cut runs). Generated on the host with a
    seeded generator, so the workload does not depend on any model state."""
    g = torch.Generator().manual_seed(seed)
    rnd = lambda *s: torch.rand(*s, generator=g)  # noqa: E731
    centre = rnd(bs, 2, na) * img
    size = 4 + 296 * rnd(bs, 2, na) ** 3
    obj_c = rnd(bs, 2, objects) * img
    obj_s = 16 + 200 * rnd(bs, 2, objects) ** 2
    which = torch.randint(0, objects, (bs, 1, na), generator=g).expand(bs, 2, na)
    near = rnd(bs, 1, na) < 0.5
    centre = torch.where(near, obj_c.gather(2, which) + 8 * (rnd(bs, 2, na) - 0.5), centre)
    size = torch.where(near, obj_s.gather(2, which) * (0.9 + 0.2 * rnd(bs, 2, na)), size)
    n = nc * na
    u = torch.stack([(torch.randperm(n, generator=g).float() + 0.5) / n for _ in range(bs)])
    return torch.cat((centre, size, (u ** 16).view(bs, nc, na)), 1)


class AugSourceDataset:
    """Synthetic stand-in for a training dataset under augmentation (the reference dataset interface the mix
    transforms use: buffer, get_image_and_label, __len__; data/base.py:290-301): n BGR uint8 images with their long
    side at imgsz (as BaseDataset.load_image leaves them) and 1-8 normalised xywh boxes each."""

    SHAPES = [(1.0, 0.75), (0.625, 1.0), (1.0, 1.0), (0.78, 1.0), (1.0, 0.5625), (1.0, 0.906), (0.5, 1.0),
              (0.875, 0.875)]

    def __init__(self, n: int, imgsz: int, seed: int = 0):
        import numpy as np

        from .instance import Instances
        self._I = Instances
        g = torch.Generator().manual_seed(seed)
        self.items = []
        for i in range(n):
            fh, fw = self.SHAPES[i % len(self.SHAPES)]
            h, w = max(8, int(round(imgsz * fh))), max(8, int(round(imgsz * fw)))
            img = torch.randint(0, 256, (h, w, 3), generator=g, dtype=torch.uint8).numpy()
            k = int(torch.randint(1, 9, (1,), generator=g))
            ctr = 0.1 + 0.8 * torch.rand(k, 2, generator=g)
            wh = torch.minimum(0.05 + 0.45 * torch.rand(k, 2, generator=g), 2 * torch.minimum(ctr, 1 - ctr))
            self.items.append({"img": img, "cls": torch.randint(0, 80, (k, 1), generator=g).float().numpy(),
                               "bboxes": torch.cat((ctr, wh), 1).numpy().astype(np.float32)})
        self.imgsz = imgsz
        self.buffer = list(range(n))
        self.data = {"flip_idx": []}
        self.use_keypoints = False

    def __len__(self):
        return len(self.items)

    def get_image_and_label(self, i):
        import numpy as np
        it = self.items[i]
        h, w = it["img"].shape[:2]
        return {"im_file": f"syn{i}.jpg", "ori_shape": (h, w), "resized_shape": (h, w), "ratio_pad": (1.0, 1.0),
                "img": it["img"], "cls": it["cls"].copy(),
                "instances": self._I(it["bboxes"].copy(), np.zeros((0, 1000, 2), dtype=np.float32), None,
                                     bbox_format="xywh", normalized=True)}
