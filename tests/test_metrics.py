"""Validator metrics tail (adrefine/utils/metrics.py) vs the reference fixture (tests/golden/metrics_val.npz, made by
oracle/gen_golden.py --only=metrics from the reference's box_iou, match_predictions, ap_per_class and Metric).
CPU: the host half (ap_per_class / Metric) on the fixture's own TP matrix. GPU: the whole tail — HIP IoU matrix,
greedy matching, AP — from the stored detections and labels."""
import numpy as np
import pytest
import torch

from conftest import golden


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
