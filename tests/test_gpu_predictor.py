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


def test_predictor_configs1_real_batch():
    """BASELINE configs[1] at its real shape: bs 32, 640x640, bf16, uint8 input (validator.py:170-190 feeds the model
    the dataloader's batch; ops.py:163-312 NMS). Graph-replayed == eager == non_max_suppression(model(x / 255))
    exactly, at the validator's settings (conf 0.001, multi-label: the max_nms cut runs) and the predictor's (conf
    0.25), with detections present on the fixed seeded recipe model."""
    from adrefine.data.synthetic import images_u8
    from adrefine.engine.predictor import FusedPredictor
    from adrefine.utils.ops import non_max_suppression
    m = _model(torch.bfloat16)
    x = images_u8(32, 640, seed=11).cuda()
    with torch.no_grad():
        y, _ = m(x.float() / 255)
    for conf, multi in ((0.001, True), (0.25, False)):
        ref = non_max_suppression(y, conf, 0.7, multi_label=multi)
        p = FusedPredictor(m, conf=conf, iou=0.7, multi_label=multi)
        eager = p.predict(x)
        p.capture(x)
        graph = p.predict(x)
        assert len(eager) == len(graph) == len(ref) == 32
        for a, b, c in zip(eager, graph, ref):
            assert a.shape == c.shape and torch.equal(a, c) and torch.equal(b, c)
        if multi:
            assert sum(len(r) for r in ref) > 0


def test_predictor_recovers_after_barrier_timeout():
    """adr_nms reports a grid-barrier timeout as -1 counts (sticky CTL_ERR control word). predict() raises, resets the
    workspace IN PLACE (same buffer: the captured hipGraph keeps writing into it) and the next replay is correct.
    The timeout is forced by setting the error word the barrier's bounded wait would set (word 2 of the workspace's
    control words, adr_nms.hip CTL_ERR)."""
    from adrefine.data.synthetic import images_u8
    from adrefine.engine.predictor import FusedPredictor
    from adrefine.utils import ops
    m = _model(torch.bfloat16)
    x = images_u8(4, 320, seed=3).cuda()
    p = FusedPredictor(m, conf=0.001, iou=0.7, multi_label=True)
    p.capture(x)
    good = p.predict(x)
    assert sum(len(r) for r in good) > 0
    dev = x.device
    ws = ops._WS[dev]
    ptr = ws.data_ptr()
    ws[:64].view(torch.int32)[2] = 1  # CTL_ERR, as a barrier wait that ran out of spins leaves it
    with pytest.raises(RuntimeError, match="grid barrier timed out"):
        p.predict(x)
    assert ops._WS[dev].data_ptr() == ptr  # not freed: the graph still references it
    assert int(ws[:64].view(torch.int32)[2]) == 0
    again = p.predict(x)
    for a, b in zip(again, good):
        assert torch.equal(a, b)
    # and the eager path on the same workspace
    ws[:64].view(torch.int32)[2] = 1
    with torch.no_grad():
        y, _ = m(x.float() / 255)
    with pytest.raises(RuntimeError):
        ops.non_max_suppression(y, 0.001, 0.7, multi_label=True)
    ref = ops.non_max_suppression(y, 0.001, 0.7, multi_label=True)
    for a, b in zip(ref, good):
        assert torch.equal(a, b)
