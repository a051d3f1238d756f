"""Validator metrics tail — drop-in for the reference's detection validation bookkeeping:
models/yolo/detect/val.py:125-229 (update_metrics, _process_batch, get_stats), engine/validator.py:221-261
(match_predictions), utils/metrics.py:52-72 (box_iou), :1054-1059 (smooth), :1112-1141 (compute_ap),
:1144-1231 (ap_per_class), :1234-1360 (Metric: mp, mr, map50, map, fitness).

Split as in the reference: the IoU matrix of each image is computed on the device (adr_box_iou, HIP), the greedy
TP matching and the AP integration run on the host in numpy, exactly as the reference does (it also moves the
IoU matrix to numpy for matching and accumulates numpy statistics). Boxes are compared in the network's input
space (the reference's scale_boxes to the original image is the identity for unpadded, unresized inputs; callers
with letterboxed images scale both sides first).
"""
from __future__ import annotations


import numpy as np
import torch

from .. import kernels as K
from ..native import lib

IOUV = np.linspace(0.5, 0.95, 10)


def box_iou(box1: torch.Tensor, box2: torch.Tensor, eps=1e-7) -> torch.Tensor:
    """(N, 4) x (M, 4) xyxy -> (N, M) IoU on the device (adr_box_iou; utils/metrics.py:52-72)."""
    if not box1.is_cuda:
        raise RuntimeError("box_iou: device tensors required (HIP kernel, no CPU fallback)")
    a = box1.float().contiguous()
    b = box2.float().contiguous()
    out = torch.empty(a.shape[0], b.shape[0], dtype=torch.float32, device=a.device)
    lib.adr_box_iou(K.fptr(a), a.shape[0], K.fptr(b), b.shape[0], float(eps), K.fptr(out), K.stream())
    return out


def match_predictions(pred_classes, true_classes, iou, iouv=IOUV):
    """engine/validator.py:221-261 (greedy, use_scipy=False): (N, 10) bool of correct detections."""
    correct = np.zeros((pred_classes.shape[0], iouv.shape[0])).astype(bool)
    correct_class = true_classes[:, None] == pred_classes
    iou = iou * correct_class
    iou = iou.cpu().numpy()
    for i, threshold in enumerate(iouv.tolist()):
        matches = np.nonzero(iou >= threshold)
        matches = np.array(matches).T
        if matches.shape[0]:
            if matches.shape[0] > 1:
                matches = matches[iou[matches[:, 0], matches[:, 1]].argsort()[::-1]]
                matches = matches[np.unique(matches[:, 1], return_index=True)[1]]
                matches = matches[np.unique(matches[:, 0], return_index=True)[1]]
            correct[matches[:, 1].astype(int), i] = True
    return correct


def smooth(y, f=0.05):
    """utils/metrics.py:1054-1059: box filter of fraction f."""
    nf = round(len(y) * f * 2) // 2 + 1
    p = np.ones(nf // 2)
    yp = np.concatenate((p * y[0], y, p * y[-1]), 0)
    return np.convolve(yp, np.ones(nf) / nf, mode="valid")


def compute_ap(recall, precision):
    """utils/metrics.py:1112-1141: COCO 101-point interpolated AP."""
    mrec = np.concatenate(([0.0], recall, [1.0]))
    mpre = np.concatenate(([1.0], precision, [0.0]))
    mpre = np.flip(np.maximum.accumulate(np.flip(mpre)))
    x = np.linspace(0, 1, 101)
    trapz = getattr(np, "trapezoid", None) or np.trapz
    ap = trapz(np.interp(x, mrec, mpre), x)
    return ap, mpre, mrec


def ap_per_class(tp, conf, pred_cls, target_cls, eps=1e-16):
    """utils/metrics.py:1144-1231 (no plotting): (tp, fp, p, r, f1, ap, unique_classes, p_curve, r_curve,
    f1_curve, x)."""
    i = np.argsort(-conf)
    tp, conf, pred_cls = tp[i], conf[i], pred_cls[i]
    unique_classes, nt = np.unique(target_cls, return_counts=True)
    nc = unique_classes.shape[0]
    x = np.linspace(0, 1, 1000)
    ap, p_curve, r_curve = np.zeros((nc, tp.shape[1])), np.zeros((nc, 1000)), np.zeros((nc, 1000))
    for ci, c in enumerate(unique_classes):
        i = pred_cls == c
        n_l = nt[ci]
        n_p = i.sum()
        if n_p == 0 or n_l == 0:
            continue
        fpc = (1 - tp[i]).cumsum(0)
        tpc = tp[i].cumsum(0)
        recall = tpc / (n_l + eps)
        r_curve[ci] = np.interp(-x, -conf[i], recall[:, 0], left=0)
        precision = tpc / (tpc + fpc)
        p_curve[ci] = np.interp(-x, -conf[i], precision[:, 0], left=1)
        for j in range(tp.shape[1]):
            ap[ci, j], _, _ = compute_ap(recall[:, j], precision[:, j])
    f1_curve = 2 * p_curve * r_curve / (p_curve + r_curve + eps)
    i = smooth(f1_curve.mean(0), 0.1).argmax()
    p, r, f1 = p_curve[:, i], r_curve[:, i], f1_curve[:, i]
    tp = (r * nt).round()
    fp = (tp / (p + eps) - tp).round()
    return tp, fp, p, r, f1, ap, unique_classes.astype(int), p_curve, r_curve, f1_curve, x


class DetectionStats:
    """The detection validator's statistics (val.py:125-190, get_stats :192-201) and box Metric
    (metrics.py:1234-1360): update(preds, batch) per batch, results() at the end."""

    def __init__(self, nc=80):
        self.nc = nc
        self.stats = {"tp": [], "conf": [], "pred_cls": [], "target_cls": [], "target_img": []}
        self.seen = 0

    def update(self, preds, batch_idx, cls, bboxes_xyxy):
        """preds: per image (n, 6) [x1, y1, x2, y2, conf, cls] device tensors (adr_nms output); labels: the batch's
        batch_idx (N,), cls (N,), xyxy boxes in input pixels (N, 4)."""
        for si, pred in enumerate(preds):
            self.seen += 1
            sel = batch_idx == si
            tcls, tbox = cls[sel], bboxes_xyxy[sel]
            npr = len(pred)
            st = {"conf": np.zeros(0), "pred_cls": np.zeros(0), "tp": np.zeros((npr, 10), dtype=bool),
                  "target_cls": tcls.cpu().numpy(), "target_img": np.unique(tcls.cpu().numpy())}
            if npr == 0:
                if len(tcls):
                    for k in self.stats:
                        self.stats[k].append(st[k])
                continue
            st["conf"] = pred[:, 4].cpu().numpy()
            st["pred_cls"] = pred[:, 5].cpu().numpy()
            if len(tcls):
                iou = box_iou(tbox.to(pred.device), pred[:, :4])
                st["tp"] = match_predictions(pred[:, 5], tcls.to(pred.device).float(), iou)
            for k in self.stats:
                self.stats[k].append(st[k])

    def results(self):
        s = {k: np.concatenate(v, 0) if v else np.zeros(0) for k, v in self.stats.items()}
        out = {"p": np.zeros(0), "r": np.zeros(0), "ap": np.zeros((0, 10)), "ap_class_index": np.zeros(0, int)}
        if len(s["tp"]) and s["tp"].any():
            _, _, p, r, _, ap, cls_idx, *_ = ap_per_class(s["tp"], s["conf"], s["pred_cls"], s["target_cls"])
            out = {"p": p, "r": r, "ap": ap, "ap_class_index": cls_idx}
        mp = float(out["p"].mean()) if len(out["p"]) else 0.0
        mr = float(out["r"].mean()) if len(out["r"]) else 0.0
        map50 = float(out["ap"][:, 0].mean()) if len(out["ap"]) else 0.0
        map_ = float(out["ap"].mean()) if len(out["ap"]) else 0.0
        fitness = float((np.array([mp, mr, map50, map_]) * [0.0, 0.0, 0.9, 0.1]).sum())
        out.update({"metrics/precision(B)": mp, "metrics/recall(B)": mr, "metrics/mAP50(B)": map50,
                    "metrics/mAP50-95(B)": map_, "fitness": fitness})
        return out
