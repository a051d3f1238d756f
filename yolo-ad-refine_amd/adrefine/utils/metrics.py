"""Validator metrics tail — drop-in for the reference's detection validation bookkeeping:
models/yolo/detect/val.py:125-229 (update_metrics, _process_batch, get_stats), engine/validator.py:221-261
(match_predictions), utils/metrics.py:52-72 (box_iou), :1054-1059 (smooth), :1112-1141 (compute_ap),
:1144-1231 (ap_per_class), :1234-1360 (Metric: mp, mr, map50, map, fitness).

The per-image work runs on the device: the IoU matrix (adr_box_iou) and the TP matching at the ten IoU thresholds
(adr_match_predictions: each detection's best same-class label, then per label and threshold the lowest-index
detection claiming it). The dataset-level AP integration runs once on the host over the concatenated statistics, from
the definitions below (own formulation, pinned by tests/golden/metrics_val.npz which the reference itself produced).
Boxes are compared in the network's input space (the reference's scale_boxes to the original image is the identity
for unpadded, unresized inputs; callers with letterboxed images scale both sides first).
"""
from __future__ import annotations

import numpy as np
import torch

from .. import kernels as K
from ..native import lib

IOUV = np.linspace(0.5, 0.95, 10)  # the validator's mAP@0.5:0.95 thresholds (val.py:36)
_PR_POINTS = 1000  # resolution of the confidence-indexed precision / recall curves (metrics.py:1191)
_AP_POINTS = 101   # COCO interpolation points (metrics.py:1135)


def box_iou(box1: torch.Tensor, box2: torch.Tensor, eps=1e-7) -> torch.Tensor:
    """(N, 4) x (M, 4) xyxy -> (N, M) IoU on the device (adr_box_iou; utils/metrics.py:52-72)."""
    if not box1.is_cuda:
        raise RuntimeError("box_iou: device tensors required (HIP kernel, no CPU fallback)")
    a = box1.float().contiguous()
    b = box2.float().contiguous()
    out = torch.empty(a.shape[0], b.shape[0], dtype=torch.float32, device=a.device)
    lib.adr_box_iou(K.fptr(a), a.shape[0], K.fptr(b), b.shape[0], float(eps), K.fptr(out), K.stream())
    return out


_THR = {}


def match_predictions(pred_classes, true_classes, iou, iouv=IOUV):
    """engine/validator.py:221-261 (greedy): (P, T) bool of correct detections, computed by adr_match_predictions from
    the (G, P) IoU matrix of one image. Thresholds are applied in float32, as the reference's comparison of a float32
    IoU array with Python floats is.

    Limits, by design: P <= 2048 detections per image (the kernel keeps each detection's best label in LDS). The
    detections come from adr_nms, which caps max_det at 300, so this path never approaches it; a larger P raises.
    Exact IoU ties between labels go to the larger label index — what the reference's reversed ascending argsort
    gives on small inputs; numpy's sort is not stable on large ones, so tie handling there is parity unpinned (a
    documented deviation)."""
    dev = iou.device
    G, P = iou.shape
    T = len(iouv)
    if G == 0 or P == 0:
        return np.zeros((P, T), dtype=bool)
    key = (str(dev), tuple(np.asarray(iouv, dtype=np.float64).tolist()))
    thr = _THR.get(key)
    if thr is None:
        thr = torch.tensor(np.asarray(iouv, dtype=np.float32), device=dev)
        _THR[key] = thr
    io = iou.float().contiguous()
    gc = true_classes.to(dev).float().contiguous()
    pc = pred_classes.to(dev).float().contiguous()
    out = torch.empty(P, T, dtype=torch.uint8, device=dev)
    lib.adr_match_predictions(K.fptr(io), G, P, K.fptr(gc), K.fptr(pc), K.fptr(thr), T, K.fptr(out), K.stream())
    return out.cpu().numpy().astype(bool)


def box_filter(y, frac):
    """metrics.py:1054-1059: moving average over an odd window of about 2*frac of the curve, the ends extended with
    the edge values."""
    width = round(len(y) * frac * 2) // 2 + 1
    ext = np.pad(y, width // 2, mode="edge")
    return np.convolve(ext, np.full(width, 1.0 / width), mode="valid")


def interpolated_ap(recall, precision):
    """metrics.py:1112-1141. Area under the precision envelope (the running maximum of precision taken from the
    high-recall end), sampled at 101 equally spaced recall levels and integrated with the trapezoid rule. The curve is
    anchored at (recall 0, precision 1) and (recall 1, precision 0)."""
    r = np.concatenate(([0.0], recall, [1.0]))
    envelope = np.maximum.accumulate(np.concatenate(([1.0], precision, [0.0]))[::-1])[::-1]
    grid = np.linspace(0, 1, _AP_POINTS)
    v = np.interp(grid, r, envelope)
    return float(np.sum(np.diff(grid) * (v[1:] + v[:-1])) / 2.0)


def ap_per_class(tp, conf, pred_cls, target_cls, eps=1e-16):
    """metrics.py:1144-1231 (no plotting). tp (n, T) bool, conf (n,), pred_cls (n,), target_cls (m,). Returns
    (tp, fp, p, r, f1, ap, classes, p_curve, r_curve, f1_curve, x) with the reference's meaning: p / r / f1 per class
    at the single confidence that maximises the smoothed class-mean F1, ap (classes, T)."""
    rank = np.argsort(-conf)  # confidence order, same sort rule as the reference
    hits, score, klass = tp[rank], conf[rank], pred_cls[rank]
    classes, n_labels = np.unique(target_cls, return_counts=True)
    n_cls, T = classes.shape[0], tp.shape[1]
    xs = np.linspace(0, 1, _PR_POINTS)
    ap = np.zeros((n_cls, T))
    p_curve = np.zeros((n_cls, _PR_POINTS))
    r_curve = np.zeros((n_cls, _PR_POINTS))
    for k in range(n_cls):
        sel = klass == classes[k]
        n_det = int(sel.sum())
        if n_det == 0 or n_labels[k] == 0:
            continue
        true_pos = np.cumsum(hits[sel], axis=0)  # (n_det, T) integer running counts
        seen = np.arange(1, n_det + 1)[:, None]    # detections so far = TP + FP
        recall = true_pos / (n_labels[k] + eps)
        precision = true_pos / seen
        neg_score = -score[sel]  # ascending abscissa for np.interp
        r_curve[k] = np.interp(-xs, neg_score, recall[:, 0], left=0)
        p_curve[k] = np.interp(-xs, neg_score, precision[:, 0], left=1)
        for t in range(T):
            ap[k, t] = interpolated_ap(recall[:, t], precision[:, t])
    f1_curve = 2 * p_curve * r_curve / (p_curve + r_curve + eps)
    at = int(box_filter(f1_curve.mean(0), 0.1).argmax())
    p, r, f1 = p_curve[:, at], r_curve[:, at], f1_curve[:, at]
    n_tp = (r * n_labels).round()
    n_fp = (n_tp / (p + eps) - n_tp).round()
    return n_tp, n_fp, p, r, f1, ap, classes.astype(int), p_curve, r_curve, f1_curve, xs


class DetectionStats:
    """The detection validator's statistics (val.py:125-190, get_stats :192-201) and box Metric
    (metrics.py:1234-1360): update(preds, batch) per batch, results() at the end."""

    KEYS = ("tp", "conf", "pred_cls", "target_cls", "target_img")

    def __init__(self, nc=80):
        self.nc = nc
        self.stats = {k: [] for k in self.KEYS}
        self.seen = 0

    def update(self, preds, batch_idx, cls, bboxes_xyxy):
        """preds: per image (n, 6) [x1, y1, x2, y2, conf, cls] device tensors (adr_nms output); labels: the batch's
        batch_idx (N,), cls (N,), xyxy boxes in input pixels (N, 4)."""
        T = len(IOUV)
        for si, pred in enumerate(preds):
            self.seen += 1
            sel = batch_idx == si
            tcls, tbox = cls[sel], bboxes_xyxy[sel]
            tcls_np = tcls.cpu().numpy()
            n = len(pred)
            if n == 0 and not len(tcls):
                continue  # an image with neither detections nor labels adds nothing (val.py:140-145)
            row = {"target_cls": tcls_np, "target_img": np.unique(tcls_np)}
            if n == 0:
                row.update(tp=np.zeros((0, T), dtype=bool), conf=np.zeros(0), pred_cls=np.zeros(0))
            else:
                row["conf"] = pred[:, 4].cpu().numpy()
                row["pred_cls"] = pred[:, 5].cpu().numpy()
                row["tp"] = (match_predictions(pred[:, 5], tcls, box_iou(tbox.to(pred.device), pred[:, :4]))
                             if len(tcls) else np.zeros((n, T), dtype=bool))
            for k in self.KEYS:
                self.stats[k].append(row[k])

    def results(self):
        s = {k: np.concatenate(v, 0) if v else np.zeros(0) for k, v in self.stats.items()}
        p = r = np.zeros(0)
        ap, idx = np.zeros((0, len(IOUV))), np.zeros(0, int)
        if len(s["tp"]) and s["tp"].any():
            _, _, p, r, _, ap, idx, *_ = ap_per_class(s["tp"], s["conf"], s["pred_cls"], s["target_cls"])
        mean = [float(v.mean()) if len(v) else 0.0 for v in (p, r, ap[:, 0] if len(ap) else ap, ap)]
        fitness = 0.9 * mean[2] + 0.1 * mean[3]  # Metric.fitness weights (0, 0, 0.9, 0.1)
        return {"p": p, "r": r, "ap": ap, "ap_class_index": idx, "metrics/precision(B)": mean[0],
                "metrics/recall(B)": mean[1], "metrics/mAP50(B)": mean[2], "metrics/mAP50-95(B)": mean[3],
                "fitness": fitness}
