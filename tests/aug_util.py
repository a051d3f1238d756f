"""Shared pieces of the augmentation parity tests: the synthetic dataset (oracle/recipe.synthetic_aug_items) behind
the reference's dataset interface (buffer, get_image_and_label, __len__; data/base.py:290-301), the chain run with
seeded RNGs as oracle/gen_golden.py `augment_fixtures` runs the reference, and a numpy executor of an ImagePlan
built from the cv2 restatements in oracle/stubs/cv2 (test infrastructure)."""
import random
import sys
from pathlib import Path
from types import SimpleNamespace

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "oracle" / "stubs"))
import cv2 as cv2_oracle  # noqa: E402  (oracle/stubs/cv2: numpy restatement)
from recipe import AUG_HYPS, synthetic_aug_items  # noqa: E402

CONFIGS = {"aug_default_256": ("default", 256, 5, [0, 1, 2, 3]), "aug_rot_256": ("rot", 256, 9, [4, 5, 6, 7, 0, 2])}


class SynthDS:
    def __init__(self, items, imgsz, instances_cls):
        self.items, self.imgsz, self.I = items, imgsz, instances_cls
        self.buffer = list(range(len(items)))
        self.data = {"flip_idx": []}
        self.use_keypoints = False

    def __len__(self):
        return len(self.items)

    def get_image_and_label(self, i):
        it = self.items[i]
        h, w = it["img"].shape[:2]
        return {"im_file": f"syn{i}.jpg", "ori_shape": (h, w), "resized_shape": (h, w), "ratio_pad": (1.0, 1.0),
                "img": it["img"].copy(), "cls": it["cls"].copy(),
                "instances": self_instances(self.I, it["bboxes"].copy())}


def self_instances(I, bboxes):
    return I(bboxes, np.zeros((0, 1000, 2), dtype=np.float32), None, bbox_format="xywh", normalized=True)


def run_chain(name):
    """Our v8_transforms + Format on the fixture's items and seeds: (list of per-sample dicts, ds)."""
    from adrefine.data.augment import Format, v8_transforms
    from adrefine.data.instance import Instances
    hypname, imgsz, seed, order = CONFIGS[name]
    hyp = SimpleNamespace(**AUG_HYPS[hypname])
    ds = SynthDS(synthetic_aug_items(8, imgsz), imgsz, Instances)
    T = v8_transforms(ds, imgsz, hyp)
    T.append(Format(bbox_format="xywh", normalize=True, batch_idx=True, bgr=hyp.bgr))
    random.seed(seed)
    np.random.seed(seed)
    return [T(ds.get_image_and_label(i)) for i in order]


def execute_plan(p):
    """The image an ImagePlan stands for, materialised stage by stage with the numpy cv2 restatement."""
    cw, ch = p.canvas
    canvas = np.full((ch, cw, 3), 114, dtype=np.uint8)
    for src, x1a, y1a, x2a, y2a, x1b, y1b in p.tiles:
        canvas[y1a:y2a, x1a:x2a] = src[y1b:y1b + (y2a - y1a), x1b:x1b + (x2a - x1a)]
    img = canvas
    if p.M is not None:
        img = cv2_oracle.warpAffine(img, p.M, dsize=p.size, borderValue=(114, 114, 114))
    if p.lut is not None:
        hsv = cv2_oracle.bgr2hsv_u8(img)
        hsv = np.stack([p.lut[k][hsv[..., k]] for k in range(3)], -1)
        img = cv2_oracle.hsv2bgr_u8(hsv)
    if p.flip_ud:
        img = img[::-1]
    if p.flip_lr:
        img = img[:, ::-1]
    img = img.transpose(2, 0, 1)
    return np.ascontiguousarray(img[::-1] if p.rgb else img)
