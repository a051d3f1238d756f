"""Batched detection inference — the device part of the reference's predict / val loop
(engine/predictor.py:130-160 preprocess + inference, models/yolo/detect/predict.py:25-40 postprocess,
models/yolo/detect/val.py:82-99 the validator's NMS call).

One batch = the dataloader's uint8 NCHW images -> /255 (fused into the stem kernel, detect/train.py:57-59's
preprocess) -> eval forward (BatchNorm with running statistics) -> DFL decode (adr_detect_decode) ->
non_max_suppression (adr_nms). After one eager warm-up the whole chain is captured into a single hipGraph, so a
batch is one graph launch plus (for `predict`) one host read of the per-image detection counts. Letterboxing
and scale_boxes back to the source image are host-side image handling outside this path; callers feed
network-sized batches.
"""
from __future__ import annotations

import torch

from .. import kernels as K
from ..utils.ops import check_counts, non_max_suppression_padded


class FusedPredictor:
    """predict(img) -> list of (n_i, 6) [x1, y1, x2, y2, conf, cls] tensors, as ops.non_max_suppression returns.

    conf / iou / max_det default to the predictor's (cfg/default.yaml: conf 0.25, iou 0.7, max_det 300); pass the
    validator's conf=0.001, multi_label=True for mAP evaluation."""

    def __init__(self, model, conf=0.25, iou=0.7, max_det=300, agnostic=False, multi_label=False, classes=None):
        self.model = model
        self.conf, self.iou, self.max_det = conf, iou, max_det
        self.agnostic, self.multi_label, self.classes = agnostic, multi_label, classes
        self.graph = None
        self.static_in = None
        self.static_out = None
        # bf16 conv operands and the eval BatchNorm scale/shift computed once, not per batch (weights are fixed here)
        self.packs = K.PackCache(cache_bn_coefs=True)

    def sync_weights(self):
        """Repack the bf16 conv operands and recompute the eval BatchNorm coefficients after the model's weights or
        running statistics changed (e.g. between training epochs)."""
        self.packs.pack_all()
        self.packs.refresh_bn_coefs()

    def _run(self, img):
        with torch.no_grad(), K.pack_scope(self.packs):
            first = not self.packs.valid
            y = self.model(img)
            if first and self.packs.specs:
                self.packs.valid = True  # the recording forward packed every operand into the cache
            y = y[0] if isinstance(y, (list, tuple)) else y
            return non_max_suppression_padded(y, self.conf, self.iou, self.classes, self.agnostic,
                                              self.multi_label, self.max_det)

    def capture(self, img):
        """Record preprocess + forward + decode + NMS for batches shaped like `img` into one hipGraph (run one
        eager batch first so lazy caches and the NMS workspace exist)."""
        self.model.eval()
        self.static_in = img.clone()
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            self._run(self.static_in)
        torch.cuda.current_stream().wait_stream(s)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, capture_error_mode="thread_local"):
            self.static_out = self._run(self.static_in)
        self.graph = g

    def run_padded(self, img):
        """(out (B, max_det, 6), n (B,) int32) on the device, no host sync."""
        self.model.eval()
        if self.graph is not None and img.shape == self.static_in.shape and img.dtype == self.static_in.dtype:
            if img.data_ptr() != self.static_in.data_ptr():
                self.static_in.copy_(img, non_blocking=True)
            self.graph.replay()
            return self.static_out
        return self._run(img)

    def predict(self, img):
        out, n = self.run_padded(img)
        counts = n.tolist()
        check_counts(counts, out.device)
        return [out[i, :k].clone() for i, k in enumerate(counts)]

    __call__ = predict
