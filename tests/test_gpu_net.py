"""GPU parity: the whole YOLO-AD-Refine-n network (701 yaml, and the 697 Mona variant) against reference-generated
fixtures."""
import pytest
import torch

from conftest import ROOT, golden
from gpu_util import assert_close, load_recipe_into
from recipe import synthetic_images

pytestmark = pytest.mark.gpu
CFG = ROOT / "tests" / "configs" / "yolo11-701-YOLO-AD-Refine.yaml"
CFG697 = ROOT / "tests" / "configs" / "yolo11-697-newfpn+mona+AYHead+mlca3.yaml"


def _model(dtype=torch.float32, cfg=CFG):
    from adrefine.nn.tasks import DetectionModel
    m = DetectionModel(str(cfg), compute_dtype=dtype)
    load_recipe_into(m)
    return m.cuda()


@pytest.mark.parametrize("tag,S", [("701", 320), ("701", 640), ("697", 320)])
def test_eval_forward(tag, S):
    g = golden(f"net{tag}_eval_{S}")
    m = _model(cfg=CFG697 if tag == "697" else CFG).eval()
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
        r = torch.as_tensor(g[f"pred{i}"]).double()
        err, sc = float((p.detach().double().cpu() - r).abs().max()), float(r.abs().max())
        print(f"pred{i}: max|d| {err:.3e} scale {sc:.3e} -> {err / (1 + sc):.2e} of (1 + max|ref|)")
        # north_star: fp32 logits within 1e-4
        assert_close(p.float(), g[f"pred{i}"], rtol=1e-4, atol=1e-4, what=f"pred{i}")
    # BN running statistics updated with momentum 0.03 / unbiased variance, as the reference
    sd = m.state_dict()
    assert_close(sd["model.0.bn.running_mean"], g["post_model.0.bn.running_mean"], rtol=1e-4, atol=1e-5)
    assert_close(sd["model.0.bn.running_var"], g["post_model.0.bn.running_var"], rtol=1e-4, atol=1e-5)
