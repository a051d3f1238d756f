"""v8DetectionLoss drop-in (reference utils/loss.py:355-520) running the whole TAL + box/DFL/cls loss and its
gradient in libadr_hip (adr_det_loss). Call contract as the reference: loss(preds, batch) ->
(loss.sum() * batch_size, loss.detach()) with loss = [box*box_gain, cls*cls_gain, dfl*dfl_gain]."""
from __future__ import annotations

import ctypes

import numpy as np
import torch

from .. import kernels as K
from ..native import lib


def preprocess_targets(batch_idx, cls, bboxes, bs, imgsz_hw):
    """loss.py:392-408 (host side, on the dataloader's CPU tensors): (B, nmax, 5) rows [cls, x1, y1, x2, y2]
    in pixels, zero-padded. Returns a pinned CPU float tensor."""
    bi = np.asarray(batch_idx.detach().cpu() if torch.is_tensor(batch_idx) else batch_idx, dtype=np.float32).reshape(-1)
    cl = np.asarray(cls.detach().cpu() if torch.is_tensor(cls) else cls, dtype=np.float32).reshape(-1)
    bx = np.asarray(bboxes.detach().cpu() if torch.is_tensor(bboxes) else bboxes, dtype=np.float32).reshape(-1, 4)
    n = bi.shape[0]
    if n == 0:
        return torch.zeros(bs, 0, 5).pin_memory() if torch.cuda.is_available() else torch.zeros(bs, 0, 5)
    idx = bi.astype(np.int64)
    counts = np.bincount(idx, minlength=bs)
    nmax = int(counts.max())
    out = np.zeros((bs, nmax, 5), dtype=np.float32)
    h, w = float(imgsz_hw[0]), float(imgsz_hw[1])
    scale = np.array([w, h, w, h], dtype=np.float32)
    # slot of every label inside its image: a stable sort by image keeps the per-image label order of the
    # reference's boolean-mask gather (loss.py:402-406), vectorised (no per-label Python loop)
    order = np.argsort(idx, kind="stable")
    starts = np.concatenate(([0], np.cumsum(counts)[:-1]))
    slot = np.empty(n, dtype=np.int64)
    slot[order] = np.arange(n) - starts[idx[order]]
    xywh = bx * scale
    out[idx, slot, 0] = cl
    out[idx, slot, 1:3] = xywh[:, :2] - xywh[:, 2:] / 2
    out[idx, slot, 3:5] = xywh[:, :2] + xywh[:, 2:] / 2
    t = torch.from_numpy(out)
    return t.pin_memory() if torch.cuda.is_available() else t


class DetLossFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, gt, strides, nc, gains, f0, f1, f2):
        feats = [f0, f1, f2]
        vs = [K.nhwc(f) for f in feats]
        B = f0.shape[0]
        no = f0.shape[1]
        dev, dtype = f0.device, f0.dtype
        A = sum(f.shape[2] * f.shape[3] for f in feats)
        nmax = gt.shape[1]
        pk = getattr(f0, "_adr_pack", None)
        if pk is not None and all(getattr(f, "_adr_pack", None) is pk for f in feats) and pk.N == B:
            # the head's level-packed output: the gradients are the level views of one packed buffer, so the head's
            # LevelSplitFn takes them back without a copy and the backward scales them in one launch
            gbuf = pk.empty(no, dtype, dev)
            grads = [pk.view(gbuf, l) for l in range(3)]
            ctx.packed = (gbuf, pk)
        else:
            grads = [K.empty_act(B, no, f.shape[2], f.shape[3], dtype, dev) for f in feats]
            ctx.packed = None
        wsb = lib.adr_det_loss_workspace(B, nmax, A)
        ws = torch.empty(wsb // 4 + 16, dtype=torch.float32, device=dev)
        out = torch.empty(5, dtype=torch.float32, device=dev)
        gtc = gt.contiguous()
        lib.adr_det_loss(K.dcode(dtype), *[ctypes.c_void_p(v[1]) for v in vs], *[v[2] for v in vs],
                         f0.shape[2], f0.shape[3], f1.shape[2], f1.shape[3], f2.shape[2], f2.shape[3],
                         float(strides[0]), float(strides[1]), float(strides[2]), B, nc, K.fptr(gtc), nmax,
                         *[ctypes.c_void_p(g.data_ptr()) for g in grads], float(B), *[float(x) for x in gains],
                         K.fptr(out), K.fptr(ws), wsb, K.stream())
        ctx.grads = grads
        total = torch.empty((), dtype=torch.float32, device=dev)
        lib.adr_cast(K.F32, ctypes.c_void_p(out.data_ptr() + 12), K.F32, K.fptr(total), 1, K.stream())
        ctx.mark_non_differentiable(out)
        return total, out

    @staticmethod
    def backward(ctx, dloss, _dout):
        grads = ctx.grads
        if ctx.packed is not None:
            gbuf, pk = ctx.packed
            sg = K.scale(gbuf, dloss.detach().float().reshape(()), "scalar")
            return (None, None, None, None, *[pk.view(sg, l) for l in range(3)])
        scaled = [K.scale(g, dloss.detach().float().reshape(()), "scalar") for g in grads]
        return (None, None, None, None, *scaled)


class v8DetectionLoss:  # noqa: N801
    """Criterion with the reference's hyper-parameters (box 7.5, cls 0.5, dfl 1.5; TAL topk 10, alpha 0.5,
    beta 6.0; SlideLoss; CIoU/NWD ratio 0.5)."""

    def __init__(self, model, tal_topk=10):
        if tal_topk != 10:
            raise NotImplementedError("adr_det_loss implements the reference's topk=10")
        m = model.model[-1]
        h = getattr(model, "args", None)
        self.hyp = h
        self.stride = m.stride
        self.nc = m.nc
        self.no = m.nc + m.reg_max * 4
        self.reg_max = m.reg_max
        self.gains = (getattr(h, "box", 7.5) if h is not None else 7.5, getattr(h, "cls", 0.5) if h is not None else 0.5,
                      getattr(h, "dfl", 1.5) if h is not None else 1.5)

    def __call__(self, preds, batch):
        feats = preds[1] if isinstance(preds, tuple) else preds
        B = feats[0].shape[0]
        dev = feats[0].device
        imgsz = (feats[0].shape[2] * float(self.stride[0]), feats[0].shape[3] * float(self.stride[0]))
        gt = batch.get("gt")
        if gt is None:
            gt = preprocess_targets(batch["batch_idx"], batch["cls"], batch["bboxes"], B, imgsz)
        gt = gt.to(dev, non_blocking=True).float()
        total, out = DetLossFn.apply(gt, [float(s) for s in self.stride], self.nc, self.gains, *feats)
        return total, out[:3]
