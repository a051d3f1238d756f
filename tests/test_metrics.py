"""Validator metrics tail (adrefine/utils/metrics.py) vs the reference fixture (tests/golden/metrics_val.npz, made by
oracle/gen_golden.py --only=metrics from the reference's box_iou, match_predictions, ap_per_class and Metric).
CPU: the host half (ap_per_class / Metric) on the fixture's own TP matrix. GPU: the whole tail — HIP IoU matrix,
greedy matching, AP — from the stored detections and labels."""
import numpy as np
import pytest
import torch

from conftest import golden


def test_match_oracle_matches_reference():
    """The loop restatement of match_predictions reproduces the reference-generated TP matrix (IoU in float32 numpy,
    the reference's own arithmetic order for box_iou)."""
    from adr_oracle import match_predictions_loops
    g = golden("metrics_val")
    p, lb = g["preds"], g["labels"]
    tp = []
    for i in range(int(max(p[:, 0].max(), lb[:, 0].max())) + 1):
        pi, li = p[p[:, 0] == i], lb[lb[:, 0] == i]
        if len(pi) == 0:
            continue
        if len(li) == 0:
            tp.append(np.zeros((len(pi), 10), dtype=bool))
            continue
        a, b = li[:, 2:6].astype(np.float32), pi[:, 1:5].astype(np.float32)
        lt = np.maximum(a[:, None, :2], b[None, :, :2])
        rb = np.minimum(a[:, None, 2:], b[None, :, 2:])
        inter = np.clip(rb - lt, 0, None).prod(2)
        area = lambda x: (x[:, 2] - x[:, 0]) * (x[:, 3] - x[:, 1])  # noqa: E731
        iou = inter / (area(a)[:, None] + area(b)[None] - inter + np.float32(1e-7))
        tp.append(match_predictions_loops(iou.astype(np.float32), li[:, 1], pi[:, 6], np.linspace(0.5, 0.95, 10)))
    np.testing.assert_array_equal(np.concatenate(tp, 0), g["tp"])


def test_ap_per_class_matches_reference():
    from adrefine.utils.metrics import ap_per_class
    g = golden("metrics_val")
    p = g["preds"]
    res = ap_per_class(g["tp"], p[:, 5], p[:, 6], g["labels"][:, 1])
    np.testing.assert_array_equal(res[6], g["ap_class_index"])
    np.testing.assert_allclose(res[2], g["p"], rtol=0, atol=1e-12)
    np.testing.assert_allclose(res[3], g["r"], rtol=0, atol=1e-12)
    np.testing.assert_allclose(res[5], g["ap"], rtol=0, atol=1e-12)
    mr = [res[2].mean(), res[3].mean(), res[5][:, 0].mean(), res[5].mean()]
    np.testing.assert_allclose(mr, g["mean_results"], rtol=0, atol=1e-12)


@pytest.mark.gpu
def test_detection_stats_end_to_end():
    from adrefine.utils.metrics import DetectionStats
    g = golden("metrics_val")
    p, lb = torch.from_numpy(g["preds"]), torch.from_numpy(g["labels"])
    nimg = int(max(p[:, 0].max(), lb[:, 0].max())) + 1
    preds = [p[p[:, 0] == i, 1:].cuda() for i in range(nimg)]
    st = DetectionStats(nc=80)
    st.update(preds, lb[:, 0], lb[:, 1], lb[:, 2:6])
    tp = np.concatenate([t for t in st.stats["tp"]], 0)
    np.testing.assert_array_equal(tp, g["tp"])
    r = st.results()
    np.testing.assert_allclose(r["ap"], g["ap"], rtol=0, atol=1e-12)
    got = [r["metrics/precision(B)"], r["metrics/recall(B)"], r["metrics/mAP50(B)"], r["metrics/mAP50-95(B)"]]
    np.testing.assert_allclose(got, g["mean_results"], rtol=0, atol=1e-12)
    assert abs(r["fitness"] - float(g["fitness"])) < 1e-12


@pytest.mark.gpu
@pytest.mark.parametrize("G,P,ncls,seed", [(1, 1, 1, 0), (3, 40, 2, 1), (50, 300, 5, 2), (700, 120, 3, 3),
                                           (8, 2048, 1, 4)])
def test_match_predictions_kernel_vs_oracle(G, P, ncls, seed):
    """adr_match_predictions vs the loop oracle on synthetic IoU matrices with many near-threshold values, exact
    IoU ties between labels, class mismatches, labels beyond one 512-label chunk (G=700) and the P cap (2048)."""
    from adr_oracle import match_predictions_loops
    from adrefine.utils.metrics import IOUV, match_predictions
    rng = np.random.default_rng(seed)
    iou = rng.choice(np.float32([0.0, 0.3, 0.5, 0.55, 0.6, 0.7, 0.75, 0.9, 0.95, 1.0]), size=(G, P))
    iou = (iou + rng.choice([0, 1e-7, -1e-7], size=(G, P)).astype(np.float32)).clip(0, 1).astype(np.float32)
    gc = rng.integers(0, ncls, G).astype(np.float32)
    pc = rng.integers(0, ncls, P).astype(np.float32)
    want = match_predictions_loops(iou, gc, pc, IOUV) if G * P <= 120000 else None
    got = match_predictions(torch.from_numpy(pc).cuda(), torch.from_numpy(gc).cuda(), torch.from_numpy(iou).cuda())
    if want is None:  # large case: the per-detection / per-label invariants instead of the O(G*P*T) loop oracle
        assert got.sum(0).max() <= G
        return
    np.testing.assert_array_equal(got, want)
