"""Box instances of one image, as the reference's ultralytics.utils.instance.Instances keeps them for detection
(utils/instance.py:34-420): a (k, 4) float32 box array with a format tag ('xyxy' / 'xywh') and a normalised flag.
Detection only: segments are the empty (0, 1000, 2) array the detection dataset builds (data/dataset.py:225) and
keypoints are None. Every operation is the reference's numpy expression, so boxes come out bit-identical."""
from __future__ import annotations

import numpy as np


def xywh2xyxy(x):
    """utils/ops.py:412-429."""
    y = np.empty_like(x)
    xy = x[..., :2]
    wh = x[..., 2:] / 2
    y[..., :2] = xy - wh
    y[..., 2:] = xy + wh
    return y


def xyxy2xywh(x):
    """utils/ops.py:396-409."""
    y = np.empty_like(x)
    y[..., 0] = (x[..., 0] + x[..., 2]) / 2
    y[..., 1] = (x[..., 1] + x[..., 3]) / 2
    y[..., 2] = x[..., 2] - x[..., 0]
    y[..., 3] = x[..., 3] - x[..., 1]
    return y


class Instances:
    """utils/instance.py:185-420, boxes only."""

    def __init__(self, bboxes, segments=None, keypoints=None, bbox_format="xywh", normalized=True):
        b = np.asarray(bboxes)
        self.bboxes = b[None, :] if b.ndim == 1 else b
        assert self.bboxes.ndim == 2 and self.bboxes.shape[1] == 4
        self.format = bbox_format
        self.normalized = normalized
        self.segments = np.zeros((0, 1000, 2), dtype=np.float32) if segments is None else segments
        if len(self.segments) or keypoints is not None:
            raise NotImplementedError("adrefine Instances: detection boxes only (no segments / keypoints)")
        self.keypoints = None

    def convert_bbox(self, format):
        if format == self.format:
            return
        if (self.format, format) == ("xywh", "xyxy"):
            self.bboxes = xywh2xyxy(self.bboxes)
        elif (self.format, format) == ("xyxy", "xywh"):
            self.bboxes = xyxy2xywh(self.bboxes)
        else:
            raise NotImplementedError(f"box format {self.format} -> {format}")
        self.format = format

    @property
    def bbox_areas(self):
        b = self.bboxes
        return (b[:, 2] - b[:, 0]) * (b[:, 3] - b[:, 1]) if self.format == "xyxy" else b[:, 3] * b[:, 2]

    def _mul(self, scale):  # Bboxes.mul, instance.py:97-112
        for k in range(4):
            self.bboxes[:, k] *= scale[k]

    def _add(self, offset):  # Bboxes.add, instance.py:114-129
        for k in range(4):
            self.bboxes[:, k] += offset[k]

    def scale(self, scale_w, scale_h, bbox_only=False):
        self._mul((scale_w, scale_h, scale_w, scale_h))

    def denormalize(self, w, h):
        if not self.normalized:
            return
        self._mul((w, h, w, h))
        self.normalized = False

    def normalize(self, w, h):
        if self.normalized:
            return
        self._mul((1 / w, 1 / h, 1 / w, 1 / h))
        self.normalized = True

    def add_padding(self, padw, padh):
        assert not self.normalized, "you should add padding with absolute coordinates."
        self._add((padw, padh, padw, padh))

    def __getitem__(self, index):
        b = self.bboxes[index]
        return Instances(b[None] if b.ndim == 1 else b, None, None, self.format, self.normalized)

    def flipud(self, h):
        if self.format == "xyxy":
            y1, y2 = self.bboxes[:, 1].copy(), self.bboxes[:, 3].copy()
            self.bboxes[:, 1] = h - y2
            self.bboxes[:, 3] = h - y1
        else:
            self.bboxes[:, 1] = h - self.bboxes[:, 1]

    def fliplr(self, w):
        if self.format == "xyxy":
            x1, x2 = self.bboxes[:, 0].copy(), self.bboxes[:, 2].copy()
            self.bboxes[:, 0] = w - x2
            self.bboxes[:, 2] = w - x1
        else:
            self.bboxes[:, 0] = w - self.bboxes[:, 0]

    def clip(self, w, h):
        ori = self.format
        self.convert_bbox("xyxy")
        self.bboxes[:, [0, 2]] = self.bboxes[:, [0, 2]].clip(0, w)
        self.bboxes[:, [1, 3]] = self.bboxes[:, [1, 3]].clip(0, h)
        if ori != "xyxy":
            self.convert_bbox(ori)

    def remove_zero_area_boxes(self):
        good = self.bbox_areas > 0
        if not all(good):
            self.bboxes = self.bboxes[good]
        return good

    def update(self, bboxes):
        self.bboxes = bboxes

    def __len__(self):
        return len(self.bboxes)

    @classmethod
    def concatenate(cls, instances_list, axis=0):
        if len(instances_list) == 1:
            return instances_list[0]
        return cls(np.concatenate([i.bboxes for i in instances_list], axis=axis), None, None,
                   instances_list[0].format, instances_list[0].normalized)
