"""GPU parity: v8DetectionLoss (TAL + CIoU/NWD + DFL + SlideLoss) value and gradients vs reference fixtures."""
import numpy as np
import pytest
import torch

from conftest import ROOT, golden
from gpu_util import assert_close, load_recipe_into
from recipe import synthetic_images

pytestmark = pytest.mark.gpu


class _M:
    def __init__(self):
        from adrefine.nn.modules.head import AYHead
        h = AYHead(80, [128, 128, 128])
        self.model = [h]
        self.args = None


def _feats(S, bs, seed, dtype):
    gen = torch.Generator().manual_seed(seed)
    feats = [torch.randn(bs, 144, S // s, S // s, generator=gen) for s in (8, 16, 32)]
    for f in feats:
        f[:, :64] *= 2.0
    return feats, [f.to("cuda", dtype).contiguous(memory_format=torch.channels_last).requires_grad_(True)
                   for f in feats]


@pytest.mark.parametrize("S,bs", [(640, 4), (320, 4)])
def test_loss_fixture(S, bs):
    from adrefine.utils.loss import v8DetectionLoss
    g = golden(f"loss_{S}_bs{bs}")
    _, fd = _feats(S, bs, int(g["feat0_seed"][0]), torch.float32)
    crit = v8DetectionLoss(_M())
    batch = {k: torch.from_numpy(g[k]) for k in ("batch_idx", "cls", "bboxes")}
    loss, items = crit(fd, batch)
    assert_close(loss.detach(), g["loss"], rtol=1e-5, atol=1e-5, what="loss")
    assert_close(items, g["items"], rtol=1e-5, atol=1e-6, what="items")
    loss.backward()
    for i, f in enumerate(fd):
        n = float(f.grad.float().norm())
        ref = float(g[f"gfeat{i}_norm"])
        assert abs(n - ref) <= 1e-4 * ref + 1e-7, (i, n, ref)
        if g[f"gfeat{i}"].size:
            assert_close(f.grad, g[f"gfeat{i}"], rtol=1e-4, atol=1e-7, what=f"gfeat{i}")


def test_loss_bf16_close():
    from adrefine.utils.loss import v8DetectionLoss
    g = golden("loss_320_bs4")
    _, fd = _feats(320, 4, int(g["feat0_seed"][0]), torch.bfloat16)
    crit = v8DetectionLoss(_M())
    batch = {k: torch.from_numpy(g[k]) for k in ("batch_idx", "cls", "bboxes")}
    loss, items = crit(fd, batch)
    assert abs(float(loss) - float(g["loss"])) <= 0.03 * float(g["loss"])


_YAMLS = {"701": "yolo11-701-YOLO-AD-Refine.yaml", "697": "yolo11-697-newfpn+mona+AYHead+mlca3.yaml"}


@pytest.mark.parametrize("tag", ["701", "697"])
def test_network_train_step_loss_and_grads(tag):
    """Whole network (701, and the 697 Mona L10 variant with Mona dropout disabled as in its fixture): train
    fwd + loss + bwd at 320^2 bs2 vs the reference (fp32 parity mode)."""
    from adrefine.nn.tasks import DetectionModel
    g = golden(f"net{tag}_train_320")
    m = DetectionModel(str(ROOT / "tests" / "configs" / _YAMLS[tag]))
    for mm in m.modules():
        if isinstance(mm, torch.nn.Dropout):
            mm.p = 0.0
    load_recipe_into(m)
    m = m.cuda().train()
    x = synthetic_images(2, 320, seed=int(g["img_seed"])).cuda()
    batch = {"img": x, **{k: torch.from_numpy(g[k]) for k in ("batch_idx", "cls", "bboxes")}}
    loss, items = m(batch)
    assert_close(loss.detach(), g["loss"], rtol=1e-4, atol=1e-4, what="loss")
    assert_close(items, g["items"], rtol=1e-4, atol=1e-5, what="items")
    loss.backward()
    ref = dict(zip([str(k) for k in g["gn_keys"]], g["gn"]))
    params = dict(m.named_parameters())
    floor = 1e-3 * max(ref.values())
    bad = []
    for k, v in ref.items():
        mine = float(params[k].grad.norm()) if params[k].grad is not None else 0.0
        if abs(mine - v) > 2e-3 * v + floor:
            bad.append((k, mine, v))
    assert not bad, bad[:10]


@pytest.mark.parametrize("kind", ["random", "zeros", "tiny"])
def test_tal_topk_fast_path_equals_serial(kind, monkeypatch):
    """TAL top-10 (utils/tal.py select_topk_candidates): the parallel fast path (unique top-10 set) and the serial
    heap-select (ADR_TAL_TOPK_SERIAL=1, the path rows with ties at the cut take) give bitwise the same loss and
    gradients. 'random' features: COCO-shape labels at bs 8 / 640 (long positive runs -> fast path; small boxes with
    fewer than 10 positive anchors -> T = 0 ties -> serial). 'zeros': every anchor predicts the same box and score,
    so mirror-symmetric anchors tie exactly at T > 0 (the fallback on tied cuts). 'tiny': boxes shrunk 8x, so most
    rows have fewer than 10 positive align values (T = 0: the short heap simulation)."""
    from adrefine.data.synthetic import labels
    from adrefine.utils.loss import v8DetectionLoss
    S, bs = 640, 8
    _, fd = _feats(S, bs, 11, torch.float32)
    if kind == "zeros":
        fd = [torch.zeros_like(f).requires_grad_(True) for f in fd]
    batch = labels(bs, 80, seed=5)
    if kind == "tiny":
        batch["bboxes"][:, 2:] /= 8
    crit = v8DetectionLoss(_M())
    out = {}
    for ser in ("1", "0"):
        monkeypatch.setenv("ADR_TAL_TOPK_SERIAL", ser)
        for f in fd:
            f.grad = None
        loss, items = crit(fd, batch)
        loss.backward()
        out[ser] = (loss.detach().clone(), items.clone(), [f.grad.clone() for f in fd])
    assert torch.equal(out["0"][0], out["1"][0]) and torch.equal(out["0"][1], out["1"][1])
    for a, b in zip(out["0"][2], out["1"][2]):
        assert torch.equal(a, b)
    assert float(out["0"][1].abs().sum()) > 0
