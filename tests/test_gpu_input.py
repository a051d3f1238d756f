"""Input pipeline: the dataloader's uint8 batch goes straight into the network — the stem
kernels (adr_stem_conv_*_u8) and adr_image_u8_to_nhwc apply preprocess_batch's .float() / 255
(models/yolo/detect/train.py:57-59) while reading — and must give exactly what the float path gives on
img.float() / 255: forward outputs, BN statistics and the stem weight gradient, bitwise."""
import pytest
import torch

from conftest import ROOT
from gpu_util import load_recipe_into

pytestmark = pytest.mark.gpu
CFG = ROOT / "tests" / "configs" / "yolo11-701-YOLO-AD-Refine.yaml"


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
def test_uint8_batch_equals_preprocessed_float(dtype):
    from adrefine.data.synthetic import images_u8
    from adrefine.nn.tasks import DetectionModel
    u8 = images_u8(2, 320, seed=3).cuda()
    f = u8.float() / 255  # preprocess_batch (detect/train.py:59)
    outs = []
    for x in (u8, f):
        m = DetectionModel(str(CFG), compute_dtype=dtype)
        load_recipe_into(m)
        m = m.cuda().train()
        preds = m(x)
        loss = sum((p.float() ** 2).mean() for p in preds)
        loss.backward()
        torch.cuda.synchronize()
        outs.append(([p.detach().float().cpu() for p in preds], m.model[0].conv.weight.grad.cpu(),
                     m.state_dict()["model.0.bn.running_mean"].cpu()))
    (pa, ga, ra), (pb, gb, rb) = outs
    for a, b in zip(pa, pb):
        d = float((a - b).abs().max())
        assert d <= 1e-6 * float(b.abs().max()) or torch.equal(a, b), d
    assert torch.allclose(ga, gb, rtol=1e-5, atol=1e-7) and torch.equal(ra, rb)
