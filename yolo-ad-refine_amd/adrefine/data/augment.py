"""The v8 training augmentation chain (reference data/augment.py v8_transforms :2273-2335) with its pixel work on
the GPU.

The transforms keep the reference's classes, constructor arguments, RNG calls (python `random` / `np.random`, same
order, same count) and label arithmetic (numpy, bit-identical boxes through adrefine.data.instance). What they do
NOT do is touch pixels: `labels["img"]` is an ImagePlan — the recipe of the image (mosaic tiles over source images,
the warpAffine matrix, the HSV LUTs, the flips, the channel order) — and `collate_fn` renders the whole batch with
one launch of adr_augment_u8 (csrc/adr_augment.hip) straight into the uint8 (B, 3, H, W) tensor the trainer reads
(FusedTrainer takes uint8 batches, /255 in the stem). The 2s x 2s mosaic canvas, the warped and the HSV images of
the reference never exist.

Covered (detection, the default hyp of cfg/default.yaml and any degrees / translate / scale / shear / flip / HSV
gains): Mosaic (n=4, p=1), CopyPaste (p=0 or no segments), RandomPerspective (perspective 0: warpAffine), MixUp
(p=0), Albumentations (absent package: no-op, as in the reference without albumentations installed), RandomHSV,
RandomFlip, Format. Not covered (raise): LetterBox / close_mosaic (cv2.resize), warpPerspective, MixUp or
CopyPaste with p > 0, mosaic9, segments / keypoints. Source images come in resized as BaseDataset.load_image leaves
them (data/base.py:151-190); decoding and that resize stay on the host."""
from __future__ import annotations

import ctypes
import math
import random

import numpy as np
import torch

from .instance import Instances

__all__ = ["ImagePlan", "Compose", "Mosaic", "CopyPaste", "RandomPerspective", "MixUp", "Albumentations", "RandomHSV",
           "RandomFlip", "Format", "v8_transforms", "collate_fn", "render", "warp_affine_tables"]


class ImagePlan:
    """A deferred uint8 BGR HWC image (see the module docstring). Stages must come in the chain's order:
    canvas (source / mosaic) -> warp -> hsv -> flips -> channel order."""

    def __init__(self, src: np.ndarray):
        if src.dtype != np.uint8 or src.ndim != 3 or src.shape[2] != 3:
            raise ValueError("ImagePlan: sources are HWC BGR uint8 images")
        h, w = src.shape[:2]
        self.tiles = [(src, 0, 0, w, h, 0, 0)]  # (source, x1a, y1a, x2a, y2a, x1b, y1b) on the canvas
        self.canvas = (w, h)
        self.size = (w, h)  # current (w, h)
        self.M = None  # 2x3 float32 warpAffine matrix (canvas -> output)
        self.lut = None  # (3, 256) uint8
        self.flip_ud = self.flip_lr = False
        self.rgb = False

    @property
    def shape(self):
        return (self.size[1], self.size[0], 3)

    def _stage(self, ok, what):
        if not ok:
            raise NotImplementedError(f"ImagePlan: {what} out of the supported chain order")


def _plan(img):
    return img if isinstance(img, ImagePlan) else ImagePlan(np.ascontiguousarray(img))


class Compose:
    """augment.py:146-316 (call, append, insert)."""

    def __init__(self, transforms):
        self.transforms = transforms if isinstance(transforms, list) else [transforms]

    def __call__(self, data):
        for t in self.transforms:
            data = t(data)
        return data

    def append(self, transform):
        self.transforms.append(transform)

    def insert(self, index, transform):
        self.transforms.insert(index, transform)


class BaseMixTransform:
    """augment.py:318-435."""

    def __init__(self, dataset, pre_transform=None, p=0.0):
        self.dataset, self.pre_transform, self.p = dataset, pre_transform, p

    def __call__(self, labels):
        if random.uniform(0, 1) > self.p:
            return labels
        indexes = self.get_indexes()
        if isinstance(indexes, int):
            indexes = [indexes]
        mix_labels = [self.dataset.get_image_and_label(i) for i in indexes]
        if self.pre_transform is not None:
            for i, data in enumerate(mix_labels):
                mix_labels[i] = self.pre_transform(data)
        labels["mix_labels"] = mix_labels
        if "texts" in labels:
            raise NotImplementedError("multi-modal texts")
        labels = self._mix_transform(labels)
        labels.pop("mix_labels", None)
        return labels


class Mosaic(BaseMixTransform):
    """augment.py:489-865, the 2x2 mosaic (_mosaic4 :657-713, _update_labels :788-812, _cat_labels :814-864)."""

    def __init__(self, dataset, imgsz=640, p=1.0, n=4):
        assert 0 <= p <= 1.0 and n in {4, 9}
        if n != 4:
            raise NotImplementedError("Mosaic n=9 (only the 2x2 mosaic of v8_transforms)")
        super().__init__(dataset=dataset, p=p)
        self.imgsz = imgsz
        self.border = (-imgsz // 2, -imgsz // 2)
        self.n = n

    def get_indexes(self, buffer=True):
        if buffer:
            return random.choices(list(self.dataset.buffer), k=self.n - 1)
        return [random.randint(0, len(self.dataset) - 1) for _ in range(self.n - 1)]

    def _mix_transform(self, labels):
        assert labels.get("rect_shape", None) is None, "rect and mosaic are mutually exclusive."
        assert len(labels.get("mix_labels", [])), "There are no other images for mosaic augment."
        return self._mosaic4(labels)

    def _mosaic4(self, labels):
        mosaic_labels = []
        s = self.imgsz
        yc, xc = (int(random.uniform(-x, 2 * s + x)) for x in self.border)
        plan = None
        for i in range(4):
            patch = labels if i == 0 else labels["mix_labels"][i - 1]
            src = _plan(patch["img"])
            if len(src.tiles) != 1 or src.M is not None or src.lut is not None:
                raise NotImplementedError("Mosaic tiles must be untransformed source images")
            img = src.tiles[0][0]
            h, w = patch.pop("resized_shape")
            if i == 0:
                plan = ImagePlan(img)
                plan.tiles, plan.canvas, plan.size = [], (2 * s, 2 * s), (2 * s, 2 * s)
                x1a, y1a, x2a, y2a = max(xc - w, 0), max(yc - h, 0), xc, yc
                x1b, y1b, x2b, y2b = w - (x2a - x1a), h - (y2a - y1a), w, h
            elif i == 1:
                x1a, y1a, x2a, y2a = xc, max(yc - h, 0), min(xc + w, s * 2), yc
                x1b, y1b, x2b, y2b = 0, h - (y2a - y1a), min(w, x2a - x1a), h
            elif i == 2:
                x1a, y1a, x2a, y2a = max(xc - w, 0), yc, xc, min(s * 2, yc + h)
                x1b, y1b, x2b, y2b = w - (x2a - x1a), 0, w, min(y2a - y1a, h)
            else:
                x1a, y1a, x2a, y2a = xc, yc, min(xc + w, s * 2), min(s * 2, yc + h)
                x1b, y1b, x2b, y2b = 0, 0, min(w, x2a - x1a), min(y2a - y1a, h)
            # img4[y1a:y2a, x1a:x2a] = img[y1b:y2b, x1b:x2b]: numpy slice semantics (empty when reversed)
            if x2a > x1a and y2a > y1a and x2b > x1b and y2b > y1b:
                plan.tiles.append((img, x1a, y1a, x2a, y2a, x1b, y1b))
            padw, padh = x1a - x1b, y1a - y1b
            patch["img"] = img  # _update_labels reads its shape
            ins = patch["instances"]
            nh, nw = img.shape[:2]
            ins.convert_bbox(format="xyxy")
            ins.denormalize(nw, nh)
            ins.add_padding(padw, padh)
            mosaic_labels.append(patch)
        final = self._cat_labels(mosaic_labels)
        final["img"] = plan
        return final

    def _cat_labels(self, mosaic_labels):
        if len(mosaic_labels) == 0:
            return {}
        imgsz = self.imgsz * 2
        final = {
            "im_file": mosaic_labels[0]["im_file"],
            "ori_shape": mosaic_labels[0]["ori_shape"],
            "resized_shape": (imgsz, imgsz),
            "cls": np.concatenate([m["cls"] for m in mosaic_labels], 0),
            "instances": Instances.concatenate([m["instances"] for m in mosaic_labels], axis=0),
            "mosaic_border": self.border,
        }
        final["instances"].clip(imgsz, imgsz)
        good = final["instances"].remove_zero_area_boxes()
        final["cls"] = final["cls"][good]
        return final


class CopyPaste(BaseMixTransform):
    """augment.py:1631-1729: a no-op without segments or with p = 0 (the detection default)."""

    def __init__(self, dataset=None, pre_transform=None, p=0.5, mode="flip"):
        super().__init__(dataset=dataset, pre_transform=pre_transform, p=p)
        self.mode = mode

    def __call__(self, labels):
        if len(labels["instances"].segments) == 0 or self.p == 0:
            return labels
        raise NotImplementedError("CopyPaste with segments")


class MixUp(BaseMixTransform):
    """augment.py:866-949: the draw of BaseMixTransform.__call__ happens; p > 0 is not covered."""

    def __init__(self, dataset, pre_transform=None, p=0.0):
        super().__init__(dataset=dataset, pre_transform=pre_transform, p=p)

    def get_indexes(self):
        return random.randint(0, len(self.dataset) - 1)

    def _mix_transform(self, labels):
        raise NotImplementedError("MixUp with p > 0")


class Albumentations:
    """augment.py:1732-1918 without the albumentations package: `transform is None`, so no draw and no change."""

    def __init__(self, p=1.0):
        self.p, self.transform = p, None

    def __call__(self, labels):
        return labels


class RandomPerspective:
    """augment.py:951-1298 with perspective 0 (cv2.warpAffine)."""

    def __init__(self, degrees=0.0, translate=0.1, scale=0.5, shear=0.0, perspective=0.0, border=(0, 0),
                 pre_transform=None):
        self.degrees, self.translate, self.scale, self.shear = degrees, translate, scale, shear
        self.perspective, self.border, self.pre_transform = perspective, border, pre_transform

    def affine_transform(self, img, border):
        """augment.py:1016-1077: the same float32 matrices, multiplied in the same order."""
        C = np.eye(3, dtype=np.float32)
        C[0, 2] = -img.shape[1] / 2
        C[1, 2] = -img.shape[0] / 2
        P = np.eye(3, dtype=np.float32)
        P[2, 0] = random.uniform(-self.perspective, self.perspective)
        P[2, 1] = random.uniform(-self.perspective, self.perspective)
        R = np.eye(3, dtype=np.float32)
        a = random.uniform(-self.degrees, self.degrees)
        s = random.uniform(1 - self.scale, 1 + self.scale)
        R[:2] = rotation_matrix_2d(a, s)
        S = np.eye(3, dtype=np.float32)
        S[0, 1] = math.tan(random.uniform(-self.shear, self.shear) * math.pi / 180)
        S[1, 0] = math.tan(random.uniform(-self.shear, self.shear) * math.pi / 180)
        T = np.eye(3, dtype=np.float32)
        T[0, 2] = random.uniform(0.5 - self.translate, 0.5 + self.translate) * self.size[0]
        T[1, 2] = random.uniform(0.5 - self.translate, 0.5 + self.translate) * self.size[1]
        M = T @ S @ R @ P @ C
        if (border[0] != 0) or (border[1] != 0) or (M != np.eye(3)).any():
            if self.perspective:
                raise NotImplementedError("RandomPerspective with perspective != 0 (warpPerspective)")
            img._stage(img.M is None and img.lut is None and not (img.flip_ud or img.flip_lr), "warp")
            img.M = M[:2].copy()
            img.size = tuple(self.size)
        return img, M, s

    def apply_bboxes(self, bboxes, M):
        n = len(bboxes)
        if n == 0:
            return bboxes
        xy = np.ones((n * 4, 3), dtype=bboxes.dtype)
        xy[:, :2] = bboxes[:, [0, 1, 2, 3, 0, 3, 2, 1]].reshape(n * 4, 2)
        xy = xy @ M.T
        xy = (xy[:, :2] / xy[:, 2:3] if self.perspective else xy[:, :2]).reshape(n, 8)
        x = xy[:, [0, 2, 4, 6]]
        y = xy[:, [1, 3, 5, 7]]
        return np.concatenate((x.min(1), y.min(1), x.max(1), y.max(1)), dtype=bboxes.dtype).reshape(4, n).T

    def __call__(self, labels):
        if self.pre_transform and "mosaic_border" not in labels:
            raise NotImplementedError("RandomPerspective pre_transform (LetterBox: mosaic p < 1 / close_mosaic)")
        labels.pop("ratio_pad", None)
        img = _plan(labels["img"])
        cls = labels["cls"]
        instances = labels.pop("instances")
        instances.convert_bbox(format="xyxy")
        instances.denormalize(*img.shape[:2][::-1])
        border = labels.pop("mosaic_border", self.border)
        self.size = img.shape[1] + border[1] * 2, img.shape[0] + border[0] * 2
        img, M, scale = self.affine_transform(img, border)
        bboxes = self.apply_bboxes(instances.bboxes, M)
        new_instances = Instances(bboxes, None, None, bbox_format="xyxy", normalized=False)
        new_instances.clip(*self.size)
        instances.scale(scale_w=scale, scale_h=scale, bbox_only=True)
        i = self.box_candidates(box1=instances.bboxes.T, box2=new_instances.bboxes.T, area_thr=0.10)
        labels["instances"] = new_instances[i]
        labels["cls"] = cls[i]
        labels["img"] = img
        labels["resized_shape"] = img.shape[:2]
        return labels

    @staticmethod
    def box_candidates(box1, box2, wh_thr=2, ar_thr=100, area_thr=0.1, eps=1e-16):
        w1, h1 = box1[2] - box1[0], box1[3] - box1[1]
        w2, h2 = box2[2] - box2[0], box2[3] - box2[1]
        ar = np.maximum(w2 / (h2 + eps), h2 / (w2 + eps))
        return (w2 > wh_thr) & (h2 > wh_thr) & (w2 * h2 / (w1 * h1 + eps) > area_thr) & (ar < ar_thr)


def rotation_matrix_2d(angle, scale):
    """cv2.getRotationMatrix2D(center=(0, 0), angle, scale) in double (imgwarp.cpp: angle *= CV_PI/180)."""
    a = angle * (math.pi / 180)
    alpha, beta = math.cos(a) * scale, math.sin(a) * scale
    return np.array([[alpha, beta, 0.0], [-beta, alpha, 0.0]], dtype=np.float64)


class RandomHSV:
    """augment.py:1301-1378: the gains and LUTs as the reference computes them; pixels on the GPU."""

    def __init__(self, hgain=0.5, sgain=0.5, vgain=0.5):
        self.hgain, self.sgain, self.vgain = hgain, sgain, vgain

    def __call__(self, labels):
        img = _plan(labels["img"])
        if self.hgain or self.sgain or self.vgain:
            r = np.random.uniform(-1, 1, 3) * [self.hgain, self.sgain, self.vgain] + 1
            x = np.arange(0, 256, dtype=r.dtype)
            lut_hue = ((x * r[0]) % 180).astype(np.uint8)
            lut_sat = np.clip(x * r[1], 0, 255).astype(np.uint8)
            lut_val = np.clip(x * r[2], 0, 255).astype(np.uint8)
            img._stage(img.lut is None and not (img.flip_ud or img.flip_lr), "hsv")
            img.lut = np.stack([lut_hue, lut_sat, lut_val])
        labels["img"] = img
        return labels


class RandomFlip:
    """augment.py:1381-1472 (boxes; no keypoints)."""

    def __init__(self, p=0.5, direction="horizontal", flip_idx=None):
        assert direction in {"horizontal", "vertical"} and 0 <= p <= 1.0
        self.p, self.direction, self.flip_idx = p, direction, flip_idx

    def __call__(self, labels):
        img = _plan(labels["img"])
        instances = labels.pop("instances")
        instances.convert_bbox(format="xywh")
        h, w = img.shape[:2]
        h = 1 if instances.normalized else h
        w = 1 if instances.normalized else w
        if self.direction == "vertical" and random.random() < self.p:
            img.flip_ud = not img.flip_ud
            instances.flipud(h)
        if self.direction == "horizontal" and random.random() < self.p:
            img.flip_lr = not img.flip_lr
            instances.fliplr(w)
        labels["img"] = img
        labels["instances"] = instances
        return labels


class Format:
    """augment.py:1920-2100 for detection (xywh, normalised, batch_idx); the image stays a plan until collate."""

    def __init__(self, bbox_format="xywh", normalize=True, return_mask=False, return_keypoint=False,
                 return_obb=False, mask_ratio=4, mask_overlap=True, batch_idx=True, bgr=0.0):
        if return_mask or return_keypoint or return_obb:
            raise NotImplementedError("Format: detection boxes only")
        self.bbox_format, self.normalize, self.batch_idx, self.bgr = bbox_format, normalize, batch_idx, bgr

    def __call__(self, labels):
        img = _plan(labels.pop("img"))
        h, w = img.shape[:2]
        cls = labels.pop("cls")
        instances = labels.pop("instances")
        instances.convert_bbox(format=self.bbox_format)
        instances.denormalize(w, h)
        nl = len(instances)
        img.rgb = random.uniform(0, 1) > self.bgr  # _format_img: img[::-1] (BGR -> RGB) unless bgr wins
        labels["img"] = img
        labels["cls"] = torch.from_numpy(cls) if nl else torch.zeros(nl)
        labels["bboxes"] = torch.from_numpy(instances.bboxes) if nl else torch.zeros((nl, 4))
        if self.normalize:
            labels["bboxes"][:, [0, 2]] /= w
            labels["bboxes"][:, [1, 3]] /= h
        if self.batch_idx:
            labels["batch_idx"] = torch.zeros(nl)
        return labels


def v8_transforms(dataset, imgsz, hyp, stretch=False):
    """augment.py:2273-2335 (detection: no keypoints, copy_paste_mode 'flip' or p = 0)."""
    mosaic = Mosaic(dataset, imgsz=imgsz, p=hyp.mosaic)
    affine = RandomPerspective(degrees=hyp.degrees, translate=hyp.translate, scale=hyp.scale, shear=hyp.shear,
                               perspective=hyp.perspective, pre_transform=None if stretch else "LetterBox")
    pre_transform = Compose([mosaic, affine])
    if hyp.copy_paste_mode == "flip":
        pre_transform.insert(1, CopyPaste(p=hyp.copy_paste, mode=hyp.copy_paste_mode))
    else:
        pre_transform.append(CopyPaste(dataset, pre_transform=None, p=hyp.copy_paste, mode=hyp.copy_paste_mode))
    return Compose([
        pre_transform,
        MixUp(dataset, pre_transform=pre_transform, p=hyp.mixup),
        Albumentations(p=1.0),
        RandomHSV(hgain=hyp.hsv_h, sgain=hyp.hsv_s, vgain=hyp.hsv_v),
        RandomFlip(direction="vertical", p=hyp.flipud),
        RandomFlip(direction="horizontal", p=hyp.fliplr, flip_idx=None),
    ])


def warp_affine_tables(M, dsize):
    """cv::warpAffine's fixed-point source coordinates (INTER_LINEAR; imgwarp.cpp WarpAffineInvoker): the 2x3 matrix
    in double, inverted as warpAffine does, then adelta[x] = cvRound(M0*x*1024), bdelta[x] = cvRound(M3*x*1024),
    X0[y] = cvRound((M1*y + M2)*1024) + 16, Y0[y] = cvRound((M4*y + M5)*1024) + 16 (AB_BITS 10, round_delta 16);
    the kernel takes X = (X0 + adelta) >> 5 (INTER_BITS 5)."""
    m = np.asarray(M, dtype=np.float64).reshape(6).copy()
    D = m[0] * m[4] - m[1] * m[3]
    D = 1.0 / D if D != 0 else 0.0
    A11, A22 = m[4] * D, m[0] * D
    m[0], m[4] = A11, A22
    m[1] *= -D
    m[3] *= -D
    b1 = -m[0] * m[2] - m[1] * m[5]
    b2 = -m[3] * m[2] - m[4] * m[5]
    m[2], m[5] = b1, b2
    W, H = dsize
    xs, ys = np.arange(W, dtype=np.float64), np.arange(H, dtype=np.float64)
    return (np.rint(m[0] * xs * 1024).astype(np.int64), np.rint(m[3] * xs * 1024).astype(np.int64),
            np.rint((m[1] * ys + m[2]) * 1024).astype(np.int64) + 16,
            np.rint((m[4] * ys + m[5]) * 1024).astype(np.int64) + 16)


class _Tile(ctypes.Structure):
    _fields_ = [("off", ctypes.c_int64)] + [(n, ctypes.c_int) for n in ("sw", "x1a", "y1a", "x2a", "y2a", "x1b", "y1b")]


class AugDesc(ctypes.Structure):
    """adr_aug_desc (include/adr.h)."""
    _fields_ = [("tile", _Tile * 4)] + [(n, ctypes.c_int) for n in (
        "ntile", "cw", "ch", "warp", "tab_off", "lut_off", "flip_ud", "flip_lr", "rgb", "pad_")]


def render(plans, device="cuda", out=None):
    """Run adr_augment_u8 for a list of ImagePlans of one output size: returns the uint8 (B, 3, H, W) batch."""
    from ..native import lib
    from ..kernels import stream

    if ctypes.sizeof(AugDesc) != lib.adr_augment_desc_size():
        raise RuntimeError("adr_aug_desc layout mismatch between adrefine and libadr_hip")
    B = len(plans)
    W, H = plans[0].size
    if any(p.size != (W, H) for p in plans):
        raise ValueError("render: every image of a batch must have the same size")
    srcs, index = [], {}
    descs = (AugDesc * B)()
    tabs, luts = [], []
    off = ntab = 0
    for b, p in enumerate(plans):
        d = descs[b]
        if len(p.tiles) > 4:
            raise ValueError("render: at most four tiles per image")
        d.ntile = len(p.tiles)
        for k, (src, x1a, y1a, x2a, y2a, x1b, y1b) in enumerate(p.tiles):
            key = id(src)
            if key not in index:
                index[key] = off
                srcs.append(np.ascontiguousarray(src).reshape(-1))
                off += src.size
            t = d.tile[k]
            t.off, t.sw = index[key], src.shape[1]
            t.x1a, t.y1a, t.x2a, t.y2a, t.x1b, t.y1b = x1a, y1a, x2a, y2a, x1b, y1b
        d.cw, d.ch = p.canvas
        d.warp = int(p.M is not None)
        if p.M is not None:
            tab = np.concatenate(warp_affine_tables(p.M, (W, H)))
            if np.abs(tab).max() >= 2 ** 31:
                raise ValueError("render: warp coordinates out of int32 range")
            d.tab_off = ntab
            tabs.append(tab.astype(np.int32))
            ntab += tab.size
        d.lut_off = -1 if p.lut is None else 768 * len(luts)
        if p.lut is not None:
            luts.append(p.lut.reshape(-1))
        d.flip_ud, d.flip_lr, d.rgb = int(p.flip_ud), int(p.flip_lr), int(p.rgb)
    pool = torch.from_numpy(np.concatenate(srcs)).to(device, non_blocking=True)
    dd = torch.frombuffer(bytearray(descs), dtype=torch.uint8).to(device, non_blocking=True)
    tb = torch.from_numpy(np.concatenate(tabs) if tabs else np.zeros(1, np.int32)).to(device, non_blocking=True)
    lt = torch.from_numpy(np.concatenate(luts) if luts else np.zeros(1, np.uint8)).to(device, non_blocking=True)
    if out is None:
        out = torch.empty(B, 3, H, W, dtype=torch.uint8, device=device)
    lib.adr_augment_u8(ctypes.c_void_p(pool.data_ptr()), ctypes.c_void_p(dd.data_ptr()), B,
                       ctypes.c_void_p(tb.data_ptr()), ctypes.c_void_p(lt.data_ptr()), ctypes.c_void_p(out.data_ptr()),
                       H, W, stream())
    out._adr_keep = (pool, dd, tb, lt)  # the inputs live until the launch has read them (stream order)
    return out


def collate_fn(batch, device="cuda"):
    """YOLODataset.collate_fn (data/dataset.py:230-246) with the images rendered on the GPU in one launch."""
    new = {"img": render([b["img"] for b in batch], device)}
    for k in ("cls", "bboxes"):
        new[k] = torch.cat([b[k] for b in batch], 0)
    new["batch_idx"] = torch.cat([b["batch_idx"] + i for i, b in enumerate(batch)], 0)
    return new
