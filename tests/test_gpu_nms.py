"""Batched NMS on the GPU (adr_nms via adrefine.utils.ops.non_max_suppression) vs the reference's
non_max_suppression (utils/ops.py:163-312): the golden fixtures produced by the reference itself (predict,
val and tight settings over 2 x 8400 anchors x 80 classes) and the oracle on seeded edge cases. The bar is
bit-exact: the same rows (boxes, scores, classes) in the same order.

Ties: the reference truncates to max_nms with an unstable CPU argsort and feeds torchvision's stable sort;
adr_nms breaks score ties by candidate order (anchor, class). Where exact score ties straddle a decision the
reference's order is implementation-defined ("parity unpinned" for such ties); the synthetic cases below use
continuous scores so the comparison is exact."""
import numpy as np
import pytest
import torch

from conftest import golden
from oracle import adr_oracle as O
from oracle.recipe import synthetic_predictions

pytestmark = pytest.mark.gpu


def _ops():
    from adrefine.utils import ops
    return ops


def _check(out, ref):
    assert len(out) == len(ref)
    for i, (o, r) in enumerate(zip(out, ref)):
        o = o.cpu().numpy()
        r = r.numpy() if isinstance(r, torch.Tensor) else r
        assert o.shape == r.shape, (i, o.shape, r.shape)
        assert np.array_equal(o, r), f"image {i}: first mismatch row {np.argwhere((o != r).any(1))[:1].ravel()}"


@pytest.mark.parametrize("name", ["predict", "val", "tight"])
def test_nms_golden(name):
    g = golden(f"nms_{name}")
    pred = synthetic_predictions(2, 8400, 80, 640, seed=7).cuda()
    out = _ops().non_max_suppression(pred, float(g["conf"]), float(g["iou"]), multi_label=bool(g["multi_label"]),
                                     max_det=300)
    _check(out, [g["out0"], g["out1"]])


CASES = [
    # (bs, na, nc, conf, iou, multi, extra kwargs)
    (3, 37, 5, 0.25, 0.45, False, {}),                    # ragged anchor count
    (2, 500, 1, 0.001, 0.7, True, {}),                    # nc == 1 disables multi_label
    (2, 1200, 20, 0.001, 0.6, True, {"max_nms": 700}),     # max_nms truncation (radix select)
    (2, 1200, 20, 0.05, 0.5, False, {"max_det": 7}),       # max_det cut across classes
    (2, 800, 12, 0.2, 0.5, False, {"classes": [0, 3, 11]}),  # classes filter
    (2, 800, 12, 0.2, 0.5, False, {"agnostic": True}),     # class-agnostic
    (2, 300, 8, 0.999, 0.5, False, {}),                    # nothing survives conf
    (4, 2100, 80, 0.25, 0.7, False, {}),                   # 320^2 grid
]


@pytest.mark.parametrize("bs,na,nc,conf,iou,multi,kw", CASES)
def test_nms_oracle(bs, na, nc, conf, iou, multi, kw):
    pred = synthetic_predictions(bs, na, nc, 640, seed=na + nc)
    ref = O.non_max_suppression(pred.clone(), conf, iou, multi_label=multi, **kw)
    out = _ops().non_max_suppression(pred.cuda(), conf, iou, multi_label=multi, **kw)
    _check(out, ref)


def test_nms_padded_no_sync_matches_list():
    pred = synthetic_predictions(2, 8400, 80, 640, seed=7).cuda()
    ops = _ops()
    out, n = ops.non_max_suppression_padded(pred, 0.25, 0.7)
    lst = ops.non_max_suppression(pred, 0.25, 0.7)
    for i, o in enumerate(lst):
        assert int(n[i]) == o.shape[0]
        assert torch.equal(out[i, : o.shape[0]], o)
        assert not out[i, o.shape[0]:].any()


def test_nms_rejects_cpu_and_unsupported():
    ops = _ops()
    pred = synthetic_predictions(1, 64, 4, 640, seed=3)
    with pytest.raises(RuntimeError):
        ops.non_max_suppression(pred)  # CPU tensor: no fallback
    with pytest.raises(NotImplementedError):
        ops.non_max_suppression(pred.cuda(), multi_label=True, agnostic=True)
