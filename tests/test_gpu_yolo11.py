"""GPU parity for config 1 (stock yolo11n: C2PSA attention, nn.Upsample, Concat, Detect) and the config-5 model
(701 yaml at scale 'l'), against reference-generated fixtures (oracle/gen_golden.py yolo11 / lscale)."""
import pytest
import torch
import torch.nn.functional as F
import yaml

from conftest import ROOT, golden
from gpu_util import assert_close, load_recipe_into
from recipe import synthetic_images

pytestmark = pytest.mark.gpu
CFG = ROOT / "tests" / "configs"


def _y11n(dtype=torch.float32):
    from adrefine.nn.tasks import DetectionModel
    m = DetectionModel(str(CFG / "yolo11n.yaml"), compute_dtype=dtype)
    load_recipe_into(m)
    return m.cuda()


def _l701(dtype=torch.float32):
    from adrefine.nn.tasks import DetectionModel
    d = yaml.safe_load((CFG / "yolo11-701-YOLO-AD-Refine.yaml").read_text())
    d["scale"] = "l"
    m = DetectionModel(d, compute_dtype=dtype)
    load_recipe_into(m)
    return m.cuda()


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("s", [2, 3])
def test_upsample_nearest(dtype, s):
    """nn.Upsample(None, s, 'nearest') forward/backward vs torch's own kernel (exact: a copy and a sum of s*s
    terms), including writing straight into a concat slice."""
    from adrefine import kernels as K
    x = torch.randn(2, 40, 7, 9, device="cuda").to(dtype).contiguous(memory_format=torch.channels_last)
    x.requires_grad_(True)
    y = K.upsample_nearest(x, s)
    ref = F.interpolate(x.detach().float(), scale_factor=s, mode="nearest")
    assert torch.equal(y.float(), ref)
    gy = torch.randn_like(ref).to(dtype).contiguous(memory_format=torch.channels_last)
    y.backward(gy)
    gref = F.avg_pool2d(gy.float(), s, s) * (s * s)
    assert torch.allclose(x.grad.float(), gref, rtol=1e-2 if dtype == torch.bfloat16 else 1e-6, atol=1e-5)
    buf = torch.zeros(2, 48, 7 * s, 9 * s, device="cuda", dtype=dtype).contiguous(memory_format=torch.channels_last)
    K.upsample_nearest(x.detach(), s, out=buf[:, 8:])
    assert torch.equal(buf[:, 8:].float(), ref) and not buf[:, :8].any()


@pytest.mark.parametrize("S", [320, 640])
def test_yolo11n_eval(S):
    g = golden(f"y11n_eval_{S}")
    m = _y11n().eval()
    x = synthetic_images(1, S, seed=int(g["img_seed"])).cuda()
    with torch.no_grad():
        y, feats = m(x)
    ref = torch.as_tensor(g["y"])
    assert_close(y[:, :4], ref[:, :4], rtol=1e-4, atol=1e-3, what="boxes")
    assert_close(y[:, 4:], ref[:, 4:], rtol=1e-4, atol=1e-4, what="scores")


def _train_check(m, g, S, loss_rtol=1e-4, gn_rtol=2e-3):
    x = synthetic_images(2, S, seed=int(g["img_seed"])).cuda()
    preds = m.train().predict(x)
    for i, p in enumerate(preds):
        assert_close(p.float(), g[f"pred{i}"], rtol=2e-4, atol=2e-4, what=f"pred{i}")
    batch = {"img": x, **{k: torch.from_numpy(g[k]) for k in ("batch_idx", "cls", "bboxes")}}
    loss, items = m.loss(batch, preds)
    assert_close(loss.detach(), g["loss"], rtol=loss_rtol, atol=1e-4, what="loss")
    assert_close(items, g["items"], rtol=loss_rtol, atol=1e-5, what="items")
    loss.backward()
    ref = dict(zip([str(k) for k in g["gn_keys"]], g["gn"]))
    params = dict(m.named_parameters())
    floor = 1e-3 * max(ref.values())
    bad = [(k, float(params[k].grad.norm()) if params[k].grad is not None else 0.0, v) for k, v in ref.items()
           if abs((float(params[k].grad.norm()) if params[k].grad is not None else 0.0) - v) > gn_rtol * v + floor]
    assert not bad, bad[:10]
    sd = m.state_dict()
    assert_close(sd["model.0.bn.running_mean"], g["post_model.0.bn.running_mean"], rtol=1e-4, atol=1e-5)
    assert_close(sd["model.0.bn.running_var"], g["post_model.0.bn.running_var"], rtol=1e-4, atol=1e-5)


def test_yolo11n_train_step():
    """Config 1 train step at 320^2 bs2 (fp32 parity mode): head outputs, loss, items, every parameter's
    gradient norm, BN running statistics."""
    _train_check(_y11n(), golden("y11n_train_320"), 320)


def test_yolo11n_bf16_train_step():
    """The same step in bf16 (performance mode). bf16 alone moves a random-recipe loss by a few percent (see
    test_gpu_bf16), so the bound is stated against the ideal-bf16 restatement (tests/bf16_sim.py: the CPU oracle
    with every functional op's output rounded to bf16) computed here: the HIP loss lies within 1.5x the ideal
    restatement's divergence from the fp32 fixture + 1 %, and never more than 3 % away unless the ideal one is."""
    import adr_oracle as O
    from bf16_sim import oracle_forward
    from conftest import state_dict_spec
    from recipe import recipe_state_dict
    g = golden("y11n_train_320")
    x = synthetic_images(2, 320, seed=int(g["img_seed"]))
    lab = {k: torch.from_numpy(g[k]) for k in ("batch_idx", "cls", "bboxes")}
    P = recipe_state_dict([(k, s) for k, s, _ in state_dict_spec("y11n")])
    with torch.no_grad():
        d = yaml.safe_load((CFG / "yolo11.yaml").read_text())
        d["scale"] = "n"
        sp = oracle_forward(P, d, x, train=True, bf16=True)
        sloss, _ = O.detection_loss(sp, lab["batch_idx"], lab["cls"], lab["bboxes"])
    ref = float(g["loss"])
    sim_dl = abs(float(sloss) - ref) / ref
    m = _y11n(torch.bfloat16).train()
    loss, items = m({"img": x.cuda(), **lab})
    dl = abs(float(loss) - ref) / ref
    print(f"loss rel: HIP bf16 {dl:.4f}, ideal bf16 {sim_dl:.4f}")
    assert dl <= max(0.03, 1.5 * sim_dl + 0.01), (dl, sim_dl)
    loss.backward()
    assert all(torch.isfinite(p.grad).all() for p in m.parameters() if p.grad is not None)


def test_701_l_eval_256():
    """Config 5's model (701 yaml, scale l: C3k2 c3k=True, C2PTSSA 256 ch / 4 heads, AYHead hidc 512) eval."""
    g = golden("net701l_eval_256")
    m = _l701().eval()
    x = synthetic_images(1, 256, seed=int(g["img_seed"])).cuda()
    with torch.no_grad():
        y, _ = m(x)
    ref = torch.as_tensor(g["y"])
    assert_close(y[:, :4], ref[:, :4], rtol=1e-4, atol=1e-3, what="boxes")
    assert_close(y[:, 4:], ref[:, 4:], rtol=1e-4, atol=1e-4, what="scores")


def test_701_l_train_step_256():
    m = _l701()
    for mm in m.modules():
        if isinstance(mm, torch.nn.Dropout):
            mm.p = 0.0
    _train_check(m, golden("net701l_train_256"), 256)
