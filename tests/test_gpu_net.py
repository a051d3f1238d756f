"""GPU parity: the whole YOLO-AD-Refine-n network (701 yaml) against reference-generated fixtures."""
import pytest
import torch

from conftest import ROOT, golden
from gpu_util import assert_close, load_recipe_into
from recipe import synthetic_images

pytestmark = pytest.mark.gpu
CFG = ROOT / "tests" / "configs" / "yolo11-701-YOLO-AD-Refine.yaml"


def _model(dtype=torch.float32):
    from adrefine.nn.tasks import DetectionModel
    m = DetectionModel(str(CFG), compute_dtype=dtype)
    load_recipe_into(m)
    return m.cuda()


@pytest.mark.parametrize("S", [320, 640])
def test_eval_forward(S):
    g = golden(f"net701_eval_{S}")
    m = _model().eval()
    x = synthetic_images(1, S, seed=int(g["img_seed"])).cuda()
    with torch.no_grad():
        y, feats = m(x)
    # boxes are in pixels (scale ~S), class scores in [0, 1]
    ref = torch.as_tensor(g["y"])
    assert_close(y[:, :4], ref[:, :4], rtol=1e-4, atol=1e-3, what="boxes")
    assert_close(y[:, 4:], ref[:, 4:], rtol=1e-4, atol=1e-4, what="scores")


def test_train_forward_head_outputs():
    g = golden("net701_train_320")
    m = _model().train()
    x = synthetic_images(2, 320, seed=int(g["img_seed"])).cuda()
    preds = m(x)
    for i, p in enumerate(preds):
        assert_close(p.float(), g[f"pred{i}"], rtol=2e-4, atol=2e-4, what=f"pred{i}")
    # BN running statistics updated with momentum 0.03 / unbiased variance, as the reference
    sd = m.state_dict()
    assert_close(sd["model.0.bn.running_mean"], g["post_model.0.bn.running_mean"], rtol=1e-4, atol=1e-5)
    assert_close(sd["model.0.bn.running_var"], g["post_model.0.bn.running_var"], rtol=1e-4, atol=1e-5)
