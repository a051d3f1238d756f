"""Restatement of torchvision.ops.nms (torchvision>=0.9, unpinned: reference pyproject.toml:73).

Published algorithm (torchvision/csrc/ops/cpu/nms_kernel.cpp): order = scores.sort(descending, stable);
for each i in order not yet suppressed: keep i, suppress every later j with
IoU(i, j) = inter / (area_i + area_j - inter) > iou_threshold, areas = (x2-x1)*(y2-y1) (no +1).
Returns kept indices (int64) in descending-score order. Oracle/test infrastructure only.
"""
import torch


def nms(boxes, scores, iou_threshold):
    boxes = boxes.detach().float().cpu()
    scores = scores.detach().float().cpu()
    n = boxes.shape[0]
    if n == 0:
        return torch.zeros(0, dtype=torch.int64)
    order = torch.sort(scores, descending=True, stable=True).indices
    x1, y1, x2, y2 = boxes.unbind(1)
    areas = (x2 - x1) * (y2 - y1)
    suppressed = torch.zeros(n, dtype=torch.bool)
    keep = []
    o = order.tolist()
    for _i, i in enumerate(o):
        if suppressed[i]:
            continue
        keep.append(i)
        rest = order[_i + 1:]
        xx1 = torch.maximum(x1[i], x1[rest])
        yy1 = torch.maximum(y1[i], y1[rest])
        xx2 = torch.minimum(x2[i], x2[rest])
        yy2 = torch.minimum(y2[i], y2[rest])
        w = (xx2 - xx1).clamp(min=0)
        h = (yy2 - yy1).clamp(min=0)
        inter = w * h
        iou = inter / (areas[i] + areas[rest] - inter)
        suppressed[rest[iou > iou_threshold]] = True
    return torch.tensor(keep, dtype=torch.int64)


def batched_nms(boxes, scores, idxs, iou_threshold):
    if boxes.numel() == 0:
        return torch.zeros(0, dtype=torch.int64)
    off = idxs.to(boxes) * (boxes.max() + 1)
    return nms(boxes + off[:, None], scores, iou_threshold)
