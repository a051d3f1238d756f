"""Pin the CPU oracle (oracle/adr_oracle.py) against fixtures produced by the reference itself
(oracle/gen_golden.py, run in the build container with /root/reference importable)."""
import math

import numpy as np
import pytest
import torch
import yaml

import adr_oracle as O
from conftest import ROOT, golden, state_dict_spec
from recipe import recipe_state_dict, seeded_randn, synthetic_images, synthetic_labels, synthetic_predictions

YAMLS = {"701": ROOT / "tests" / "configs" / "yolo11-701-YOLO-AD-Refine.yaml",
         "697": ROOT / "tests" / "configs" / "yolo11-697-newfpn+mona+AYHead+mlca3.yaml",
         "y11n": ROOT / "tests" / "configs" / "yolo11.yaml",
         "701l": ROOT / "tests" / "configs" / "yolo11-701-YOLO-AD-Refine.yaml"}
SCALES = {"y11n": "n", "701l": "l"}


def _close(a, b, rtol=1e-4, atol=1e-5):
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    assert a.shape == b.shape, (a.shape, b.shape)
    err = np.abs(a - b).max() if a.size else 0.0
    scale = np.abs(b).max() if b.size else 0.0
    assert err <= atol + rtol * scale, f"max|d|={err:.3e} vs scale {scale:.3e}"


def _module_params(prefix_keys):
    return recipe_state_dict(prefix_keys)


def _mod_run(name, keys, fn):
    """Rebuild the module fixture inputs from seeds, run fn(P, inputs) -> outputs; compare fwd + input grads."""
    g = golden(f"mod_{name}")
    P = recipe_state_dict(keys)
    for k, v in P.items():
        if v.dtype.is_floating_point and "running" not in k:
            v.requires_grad_(True)
    ins = []
    i = 0
    while f"in{i}_shape" in g:
        ins.append(seeded_randn(*[int(s) for s in g[f"in{i}_shape"]], seed=int(g[f"in{i}_seed"])).requires_grad_(True))
        i += 1
    outs = fn(P, ins)
    outs = outs if isinstance(outs, (list, tuple)) else [outs]
    gen = torch.Generator().manual_seed(int(name_seed[name]) + 1)
    gouts = [torch.randn(o.shape, generator=gen) for o in outs]
    torch.autograd.backward(list(outs), gouts)
    for j, o in enumerate(outs):
        _close(o.detach(), g[f"out{j}"])
    for j, x in enumerate(ins):
        _close(x.grad, g[f"gin{j}"])
    ref = dict(zip([str(k) for k in g["param_grad_norms_keys"]], g["param_grad_norms"]))
    for k, v in ref.items():
        pg = P[k].grad
        mine = float(pg.norm()) if pg is not None else 0.0
        assert abs(mine - v) <= 1e-4 * max(1.0, abs(v)), (k, mine, v)


name_seed = {"conv_k3s2": 21, "c3k2": 22, "c3k2_mlca_c3k": 23, "c3k2_mlca": 24, "sppf": 25, "ela": 26,
             "ela_noflag": 27, "convT": 28, "fusion": 29, "c2ptssa": 30, "c2tssa_mona": 31, "ayhead": 32,
             "c2psa": 33, "c2psa_l": 34, "detect": 35}


def _keys_for(prefix, tag="701", strip=True):
    out = []
    for k, s, _ in state_dict_spec(tag):
        if k.startswith(prefix + "."):
            out.append((k[len(prefix) + 1:] if strip else k, s))
    return out


@pytest.fixture(autouse=True)
def _threads(cpu_threads):
    yield


def test_conv_module():
    keys = [("conv.weight", (32, 16, 3, 3)), ("bn.weight", (32,)), ("bn.bias", (32,)), ("bn.running_mean", (32,)),
            ("bn.running_var", (32,)), ("bn.num_batches_tracked", ())]
    _mod_run("conv_k3s2", keys, lambda P, x: O.conv_bn_act(_prefixed(P), "m", x[0], 3, 2))


def _prefixed(P):
    return {"m." + k: v for k, v in P.items()}


def test_fusion_module():
    keys = [("fusion_weight", (2,))]
    _mod_run("fusion", keys, lambda P, x: O.fusion_bifpn(_prefixed(P), "m", x))


def test_ela_modules():
    keys = [("conv1x1.0.weight", (128, 128, 7)), ("conv1x1.0.bias", (128,)), ("conv1x1.1.weight", (128,)),
            ("conv1x1.1.bias", (128,))]
    _mod_run("ela", keys, lambda P, x: O.ela_hsfpn(_prefixed(P), "m", x[0], True))
    _mod_run("ela_noflag", keys, lambda P, x: O.ela_hsfpn(_prefixed(P), "m", x[0], False))


def test_convT_module():
    keys = [("weight", (128, 128, 3, 3)), ("bias", (128,))]
    _mod_run("convT", keys, lambda P, x: torch.nn.functional.conv_transpose2d(x[0], P["weight"], P["bias"], 2, 1, 1))


def test_c3k2_modules():
    _mod_run("c3k2", _keys_for("model.2"), lambda P, x: O.c2f_family(_prefixed(P), "m", x[0], 32, 64, 1, False, 0.25,
                                                                      True, True, False))
    _mod_run("c3k2_mlca_c3k", _keys_for("model.6"),
             lambda P, x: O.c2f_family(_prefixed(P), "m", x[0], 128, 128, 1, True, 0.5, True, True, True))
    _mod_run("c3k2_mlca", _keys_for("model.19"),
             lambda P, x: O.c2f_family(_prefixed(P), "m", x[0], 128, 128, 1, False, 0.5, True, True, True))


def test_sppf_module():
    _mod_run("sppf", _keys_for("model.9"), lambda P, x: O.sppf(_prefixed(P), "m", x[0]))


def test_c2ptssa_module():
    _mod_run("c2ptssa", _keys_for("model.10"), lambda P, x: O.c2ptssa(_prefixed(P), "m", x[0], 256, 256, 1))


def test_c2tssa_mona_module():
    _mod_run("c2tssa_mona", _keys_for("model.10", "697"),
             lambda P, x: O.c2tssa_mona(_prefixed(P), "m", x[0], 256, 256, 1))


def test_ayhead_module():
    _mod_run("ayhead", _keys_for("model.33"), lambda P, x: O.ayhead(_prefixed(P), "m", x, 80, True))


def test_c2psa_modules():
    _mod_run("c2psa", _keys_for("model.10", "y11n"), lambda P, x: O.c2psa(_prefixed(P), "m", x[0], 256, 256, 1))
    from adrefine.nn.modules.block import C2PSA  # key order of the same module at 512 channels, 2 blocks
    keys = [(k, tuple(v.shape)) for k, v in C2PSA(512, 512, 2).state_dict().items()]
    _mod_run("c2psa_l", keys, lambda P, x: O.c2psa(_prefixed(P), "m", x[0], 512, 512, 2))


def test_detect_module():
    _mod_run("detect", _keys_for("model.23", "y11n"),
             lambda P, x: O.detect(_prefixed(P), "m", x, 80, True, (8, 16, 32)))


def _net(tag):
    P = recipe_state_dict([(k, s) for k, s, _ in state_dict_spec(tag)])
    d = yaml.safe_load(YAMLS[tag].read_text())
    layers, save = O.parse(d, 3, SCALES.get(tag) or O.guess_scale(YAMLS[tag].name) or None)
    return P, layers, save


def _fixture_name(tag, kind, S):
    return f"y11n_{kind}_{S}" if tag == "y11n" else f"net{tag}_{kind}_{S}"


@pytest.mark.parametrize("tag,S", [("701", 320), ("701", 640), ("697", 320), ("y11n", 320), ("y11n", 640),
                                   ("701l", 256)])
def test_net_eval(tag, S):
    g = golden(_fixture_name(tag, "eval", S))
    P, layers, save = _net(tag)
    x = synthetic_images(1, S, seed=int(g["img_seed"]))
    with torch.no_grad():
        y, _ = O.forward(P, layers, save, x, train=False)
    _close(y, g["y"], rtol=2e-5, atol=1e-4)


@pytest.mark.parametrize("tag,S", [("701", 320), ("697", 320), ("y11n", 320), ("701l", 256)])
def test_net_train_step(tag, S):
    g = golden(_fixture_name(tag, "train", S))
    P, layers, save = _net(tag)
    for k, v in P.items():
        if v.dtype.is_floating_point and "running" not in k:
            v.requires_grad_(True)
    x = synthetic_images(2, S, seed=int(g["img_seed"]))
    preds = O.forward(P, layers, save, x, train=True)
    for i, p in enumerate(preds):
        _close(p.detach(), g[f"pred{i}"], rtol=1e-4, atol=1e-4)
    loss, items = O.detection_loss(preds, torch.from_numpy(g["batch_idx"]), torch.from_numpy(g["cls"]),
                                   torch.from_numpy(g["bboxes"]))
    _close(loss.detach(), g["loss"], rtol=1e-4)
    _close(items, g["items"], rtol=1e-4, atol=1e-5)
    loss.backward()
    ref = dict(zip([str(k) for k in g["gn_keys"]], g["gn"]))
    bad = []
    for k, v in ref.items():
        mine = float(P[k].grad.norm()) if P[k].grad is not None else 0.0
        if abs(mine - v) > 2e-3 * max(abs(v), 1e-3):
            bad.append((k, mine, v))
    assert not bad, bad[:10]
    for k in ("model.0.bn.running_mean", "model.0.bn.running_var"):
        _close(P[k].detach(), g["post_" + k], rtol=1e-5, atol=1e-6)


@pytest.mark.parametrize("S,bs", [(640, 4), (320, 4)])
def test_loss_fixture(S, bs):
    g = golden(f"loss_{S}_bs{bs}")
    gen = torch.Generator().manual_seed(int(g["feat0_seed"][0]))
    feats = [torch.randn(bs, 144, S // s, S // s, generator=gen) for s in (8, 16, 32)]
    for f in feats:
        f[:, :64] *= 2.0
        f.requires_grad_(True)
    loss, items = O.detection_loss(feats, torch.from_numpy(g["batch_idx"]), torch.from_numpy(g["cls"]),
                                   torch.from_numpy(g["bboxes"]))
    _close(loss.detach(), g["loss"], rtol=1e-5)
    _close(items, g["items"], rtol=1e-5, atol=1e-6)
    loss.backward()
    for i, f in enumerate(feats):
        assert abs(float(f.grad.norm()) - float(g[f"gfeat{i}_norm"])) <= 1e-5 * float(g[f"gfeat{i}_norm"]) + 1e-7
        if g[f"gfeat{i}"].size:
            _close(f.grad, g[f"gfeat{i}"], rtol=1e-5, atol=1e-7)


@pytest.mark.parametrize("name", ["predict", "val", "tight"])
def test_nms_fixture(name):
    g = golden(f"nms_{name}")
    pred = synthetic_predictions(2, 8400, 80, 640, seed=7)
    out = O.non_max_suppression(pred, float(g["conf"]), float(g["iou"]), multi_label=bool(g["multi_label"]))
    for i, o in enumerate(out):
        ref = g[f"out{i}"]
        assert o.shape == ref.shape, (o.shape, ref.shape)
        assert np.array_equal(o.numpy(), ref), "NMS output must match bit-exactly"


def _grad_close(mine, ref, rtol):
    """max |mine - ref| <= rtol * max |ref| (elementwise, per parameter tensor)."""
    mine, ref = mine.detach().double(), torch.as_tensor(ref).double()
    return float((mine - ref).abs().max()) <= rtol * float(ref.abs().max()) + 1e-12


def test_net701_full_param_grads():
    """The oracle's full dL/dtheta for the GRAD_KEYS subset against the reference's (net701_grads_320), elementwise."""
    g = golden("net701_grads_320")
    P, layers, save = _net("701")
    for k, v in P.items():
        if v.dtype.is_floating_point and "running" not in k:
            v.requires_grad_(True)
    x = synthetic_images(2, int(g["img_size"]), seed=int(g["img_seed"]))
    preds = O.forward(P, layers, save, x, train=True)
    loss, _ = O.detection_loss(preds, torch.from_numpy(g["batch_idx"]), torch.from_numpy(g["cls"]),
                               torch.from_numpy(g["bboxes"]))
    _close(loss.detach(), g["loss"], rtol=1e-4)
    loss.backward()
    bad = [str(k) for i, k in enumerate(g["keys"]) if not _grad_close(P[str(k)].grad, g[f"g{i}"], 2e-4)]
    assert not bad, bad
