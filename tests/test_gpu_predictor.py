"""GPU: the batched inference engine (engine/predictor.py; BASELINE.json configs[1]) — uint8 batch -> eval forward ->
decode -> NMS, eager and as one hipGraph."""
import pytest
import torch

from conftest import ROOT
from gpu_util import load_recipe_into

pytestmark = pytest.mark.gpu
CFG = ROOT / "tests" / "configs" / "yolo11-701-YOLO-AD-Refine.yaml"


def _model(dtype):
    from adrefine.nn.tasks import DetectionModel
    m = DetectionModel(str(CFG), compute_dtype=dtype)
    load_recipe_into(m)
    return m.cuda().eval()


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_predictor_matches_model_plus_nms(dtype):
    """predict(uint8) == non_max_suppression(model(uint8 / 255)) exactly, eager and graph-replayed."""
    from adrefine.data.synthetic import images_u8
    from adrefine.engine.predictor import FusedPredictor
    from adrefine.utils.ops import non_max_suppression
    m = _model(dtype)
    x = images_u8(4, 320, seed=3).cuda()
    with torch.no_grad():
        y, _ = m(x.float() / 255)
    ref = non_max_suppression(y, 0.001, 0.7, multi_label=True)  # validator settings: many detections
    p = FusedPredictor(m, conf=0.001, iou=0.7, multi_label=True)
    eager = p.predict(x)
    p.capture(x)
    graph = p.predict(x)
    x2 = images_u8(4, 320, seed=4).cuda()
    graph2 = p.predict(x2)  # a new batch goes through the static input
    with torch.no_grad():
        y2, _ = m(x2.float() / 255)
    ref2 = non_max_suppression(y2, 0.001, 0.7, multi_label=True)
    for a, b, c in zip(eager, graph, ref):
        assert a.shape == c.shape and torch.equal(a, c) and torch.equal(b, c)
    for a, b in zip(graph2, ref2):
        assert torch.equal(a, b)
    assert sum(len(r) for r in ref) > 0
