"""Post-processing on the device — drop-in for the reference's ultralytics/utils/ops.py:163-312
`non_max_suppression` (the detect predict/val callers: models/yolo/detect/predict.py:25,
models/yolo/detect/val.py:94). The whole batch runs in one persistent HIP launch (adr_nms: candidate
extraction, max_nms radix select, per-class greedy NMS, max_det merge, separated by grid barriers); the only host sync is reading the per-image counts to
split the padded result into the reference's list of (n, 6) tensors."""
from __future__ import annotations

import ctypes

import torch

from ..kernels import fptr, stream
from ..native import lib

_WS = {}


def _workspace(device, nbytes):
    """adr_nms keeps its grid barrier's control words in the first 64 bytes of the workspace: zero on first use
    (the buffer is zero-filled when (re)allocated) and left zero by every call."""
    ws = _WS.get(device)
    if ws is None or ws.numel() < nbytes:
        ws = torch.zeros(nbytes, dtype=torch.uint8, device=device)
        _WS[device] = ws
    return ws


def non_max_suppression_padded(prediction, conf_thres=0.25, iou_thres=0.45, classes=None, agnostic=False,
                               multi_label=False, max_det=300, nc=0, max_nms=30000, max_wh=7680):
    """Same selection as non_max_suppression, returned without a host sync: (out (B, max_det, 6), n (B,) int32)."""
    assert 0 <= conf_thres <= 1, f"Invalid Confidence threshold {conf_thres}, valid values are between 0.0 and 1.0"
    assert 0 <= iou_thres <= 1, f"Invalid IoU {iou_thres}, valid values are between 0.0 and 1.0"
    if isinstance(prediction, (list, tuple)):  # (inference_out, loss_out) from a model in eval mode
        prediction = prediction[0]
    if not prediction.is_cuda:
        raise RuntimeError("adrefine non_max_suppression runs on a ROCm device only (got a CPU tensor)")
    if prediction.shape[-1] == 6:
        raise NotImplementedError("end-to-end (B, 300, 6) predictions are not produced on this path")
    B, ch, A = prediction.shape
    nc = nc or (ch - 4)
    if ch - 4 - nc:
        raise NotImplementedError("mask coefficients (nm > 0) are not on the detection path")
    multi = bool(multi_label and nc > 1)
    if agnostic and multi:
        raise NotImplementedError("agnostic multi-label NMS (nc > 1) is not supported by adr_nms")
    y = prediction.detach()
    if y.dtype != torch.float32 or not y.is_contiguous():
        y = y.float().contiguous()
    dev = y.device
    cmask = None
    if classes is not None:
        cmask = torch.zeros(nc, dtype=torch.uint8)
        for c in (classes.tolist() if isinstance(classes, torch.Tensor) else list(classes)):
            if 0 <= int(c) < nc:
                cmask[int(c)] = 1
        cmask = cmask.to(dev, non_blocking=False)
    out = torch.zeros(B, max_det, 6, dtype=torch.float32, device=dev)
    n = torch.zeros(B, dtype=torch.int32, device=dev)
    nbytes = int(lib.adr_nms_workspace(B, nc, A, int(multi), max_det))
    ws = _workspace(dev, nbytes)
    lib.adr_nms(fptr(y), B, nc, A, float(conf_thres), float(iou_thres), int(multi), int(bool(agnostic)),
                ctypes.c_void_p(cmask.data_ptr() if cmask is not None else 0), int(max_det), int(max_nms),
                float(max_wh), fptr(out), ctypes.c_void_p(n.data_ptr()), ctypes.c_void_p(ws.data_ptr()), nbytes,
                stream())
    return out, n


def non_max_suppression(prediction, conf_thres=0.25, iou_thres=0.45, classes=None, agnostic=False,
                        multi_label=False, labels=(), max_det=300, nc=0, max_time_img=0.05, max_nms=30000,
                        max_wh=7680, in_place=True, rotated=False):
    """ops.py:163-312. Returns a list of B tensors (n_i, 6): x1, y1, x2, y2, conf, cls.

    Differences, by design: `prediction` is not rewritten to xyxy in place (`in_place` is accepted and ignored);
    there is no wall-clock time limit (`max_time_img` ignored: the batch is one device pass); apriori `labels`
    (autolabelling), rotated boxes and mask coefficients are not on this path and raise."""
    if rotated:
        raise NotImplementedError("rotated (OBB) NMS is not on the AD-Refine detection path")
    if labels and any(len(lb) for lb in labels):
        raise NotImplementedError("apriori labels (save_hybrid autolabelling) are not on the AD-Refine path")
    out, n = non_max_suppression_padded(prediction, conf_thres, iou_thres, classes, agnostic, multi_label, max_det,
                                        nc, max_nms, max_wh)
    counts = n.tolist()
    check_counts(counts, prediction.device)
    return [out[i, :k] for i, k in enumerate(counts)]


def check_counts(counts, device):
    """A negative per-image count is adr_nms's report of a grid-barrier timeout (the persistent kernel's phases ran
    out of order). Raise, after returning the workspace to its first-use state IN PLACE (adr_nms_reset zeroes the
    control words, sticky error flag included): the buffer is not freed, because a FusedPredictor hipGraph may have
    captured adr_nms on it — freeing would let the allocator hand that memory to another tensor while the graph
    still writes into it. The next call (eager or replayed) runs from zeroed control words."""
    if any(k < 0 for k in counts):
        ws = _WS.get(device)
        if ws is not None:
            lib.adr_nms_reset(ctypes.c_void_p(ws.data_ptr()), ws.numel(), stream())
            torch.cuda.current_stream(device).synchronize()
        raise RuntimeError("adr_nms: a grid barrier timed out (workgroups not co-resident?); detections are invalid")
