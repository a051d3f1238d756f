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


@pytest.mark.parametrize("layout", ["direct", "scanned"])
@pytest.mark.parametrize("conf,multi,kw", [(0.25, False, {}), (0.001, True, {}), (0.001, True, {"max_nms": 3000}),
                                           (0.05, False, {"agnostic": True}), (0.001, False, {"max_nms": 2000})])
def test_nms_persistent_matches_chain(monkeypatch, layout, conf, multi, kw):
    """The single persistent launch (default) in both bucket layouts against the six-kernel chain
    (ADR_NMS_MODE=chain) on a full-size batch (8 x 8400 anchors x 80 classes): identical rows, also when the
    workspace holds another shape's data and when a direct launch skips its cursor-zeroing pass (second call, same
    shape); the grid barrier never timed out."""
    ops = _ops()
    if layout == "scanned":
        monkeypatch.setenv("ADR_NMS_DIRECT", "0")
    pred = synthetic_predictions(8, 8400, 80, 640, seed=11).cuda()
    out_p, n_p = ops.non_max_suppression_padded(pred, conf, 0.7, multi_label=multi, **kw)
    ops.non_max_suppression_padded(pred[:3, :, :1000].contiguous(), 0.001, 0.5, multi_label=True)  # other shape
    out_p2, n_p2 = ops.non_max_suppression_padded(pred, conf, 0.7, multi_label=multi, **kw)
    out_p3, n_p3 = ops.non_max_suppression_padded(pred, conf, 0.7, multi_label=multi, **kw)  # record reused
    torch.cuda.synchronize()
    ctl = ops._WS[pred.device][:64].view(torch.int32).cpu()
    assert int(ctl[2]) == 0, "grid barrier timed out"
    assert int(ctl[6]) == (1 if layout == "direct" else 0), "cursor record"
    monkeypatch.setenv("ADR_NMS_MODE", "chain")
    out_c, n_c = ops.non_max_suppression_padded(pred, conf, 0.7, multi_label=multi, **kw)
    assert int(n_c.sum()) > 0
    for o, n in ((out_p, n_p), (out_p2, n_p2), (out_p3, n_p3)):
        assert torch.equal(n, n_c)
        assert torch.equal(o, out_c)
